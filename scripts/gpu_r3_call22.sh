# A/B: range-table forward kernel (default build) vs HEAD's kernel (variants/lib_head.so):
# event-timed tap launches at 512^2 V=8 and short bench lines, alternating.
set -u
mkdir -p gpurun_out
for i in 1 2; do
  for lib in distributed-inverse-problem-admm_amd/admm_hip/libadmm_tomo.so variants/lib_head.so; do
    ADMM_TOMO_LIB=$lib timeout -k 10 120 python -u scripts/time_fwd.py >> gpurun_out/ab_range.txt 2>&1 || exit $?
    ADMM_TOMO_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --strong none \
      > gpurun_out/ab_bench.json 2>/dev/null || exit $?
    python - "$lib" >> gpurun_out/ab_range.txt <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_bench.json").read().strip().splitlines()[-1])
print(sys.argv[1].split("/")[-1], "bench", round(d["value"], 1), "node-updates/s", round(d["ms_per_step"], 3), "ms/step fwd",
      round(d["roofline"]["avg_launch_ms"] * 1e3, 2), "us")
PY
  done
done
cat gpurun_out/ab_range.txt
