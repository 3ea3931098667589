# Forward block size A/B: at most 16 (default), 12 or 8 angles (waves) per block -- every
# plan's event-timed tap launch at 512^2 / 1024^2, then a short bench line per build.
set -u
mkdir -p gpurun_out
for v in g16:distributed-inverse-problem-admm_amd/admm_hip/libadmm_tomo.so g12:variants/lib_g12.so g8:variants/lib_g8.so; do
  name=${v%%:*}; lib=${v#*:}
  echo "== $name" >> gpurun_out/ab_g.txt
  ADMM_TOMO_LIB=$lib SIZES=512:float32,1024:float32 timeout -k 10 300 python -u scripts/time_fwd_plans.py >> gpurun_out/ab_g.txt 2>&1 || exit $?
  ADMM_TOMO_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --strong none > gpurun_out/ab_g_bench.json 2>/dev/null || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/ab_g_bench.json').read().strip().splitlines()[-1]); print('$name bench', round(d['value'],1), round(d['ms_per_step'],3), 'fwd', round(d['roofline']['avg_launch_ms']*1e3,2))" >> gpurun_out/ab_g.txt
done
grep -v amdgpu.ids gpurun_out/ab_g.txt
