# BASELINE config lines with the six-plan picker, and two default bench lines.
set -u
mkdir -p gpurun_out
bash scripts/run_configs.sh C5s C4 C2 C3 || exit $?
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --strong none > gpurun_out/b.json 2>/dev/null || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/b.json').read().strip().splitlines()[-1]); print('bench', round(d['value'],1), round(d['ms_per_step'],3), 'fwd', round(d['roofline']['avg_launch_ms']*1e3,2), d['roofline']['fwd_plan']['plan'])"
done
