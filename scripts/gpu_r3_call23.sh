# A/B: float64 batches at node-interleave width 8 (default) vs 4 (variants/lib_f64vb4.so:
# 32-byte sample vectors -> LDS-DMA forward staging, prefetched back windows, <= 64/110
# VGPRs): forward plans at 2048^2 and the C5s config line with each.
set -u
mkdir -p gpurun_out
for lib in distributed-inverse-problem-admm_amd/admm_hip/libadmm_tomo.so variants/lib_f64vb4.so; do
  echo "== $lib" >> gpurun_out/ab_f64vb.txt
  ADMM_TOMO_LIB=$lib SIZES=2048:float64 timeout -k 10 300 python -u scripts/time_fwd_plans.py >> gpurun_out/ab_f64vb.txt 2>&1 || exit $?
  ADMM_TOMO_LIB=$lib timeout -k 10 400 python bench.py --config C5s --steps 3 --warmup 1 > gpurun_out/c5s.json 2>/dev/null || exit $?
  python -c "import json; b=json.load(open('gpurun_out/c5s.json')); print('C5s', round(b['value'],2), 'node-updates/s', round(b['ms_per_step'],1), 'ms/step fwd', round(b['roofline']['avg_launch_ms']*1e3,1), 'us')" >> gpurun_out/ab_f64vb.txt
done
cat gpurun_out/ab_f64vb.txt
