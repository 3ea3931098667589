# Forward plans with per-segment ray clipping (rays that miss the segment inside the image get
# no lanes; their zero partials stay zero): projector / ADMM / plan-bitwise parity, then the
# plans side by side and bench lines vs the unclipped build (variants/lib_noclip.so).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize_projector.py tests/test_gpu_projector.py \
  tests/test_gpu_admm.py tests/test_gpu_matrix.py -m gpu -q -x -rf --timeout 200 --timeout-method thread > gpurun_out/pytest_clip.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_clip.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/time_fwd_plans.py > gpurun_out/fwd_plans_clip.jsonl 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/fwd_plans_clip.jsonl
for i in 1 2; do
for v in clip:distributed-inverse-problem-admm_amd/admm_hip/libadmm_tomo.so noclip:variants/lib_noclip.so; do
  name=${v%%:*}; lib=${v#*:}
  ADMM_TOMO_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --strong none > gpurun_out/ab_clip.json 2>/dev/null || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/ab_clip.json').read().strip().splitlines()[-1]); print('$name bench', round(d['value'],1), round(d['ms_per_step'],3), 'fwd', round(d['roofline']['avg_launch_ms']*1e3,2), d['roofline']['fwd_plan'])"
done
done
for c in C5s C4; do
  timeout -k 10 400 python bench.py --config $c --steps 3 --warmup 1 > gpurun_out/config_$c.json 2>/dev/null || exit $?
  python -c "import json; b=json.load(open('gpurun_out/config_$c.json')); print('$c', round(b['value'],2), 'node-updates/s', round(b['ms_per_step'],1), 'ms/step fwd', round(b['roofline']['avg_launch_ms']*1e3,1), 'us')"
done
