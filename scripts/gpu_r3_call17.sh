# rocprofv3 kernel stats of the C5s (2048^2 float64) and C4 (1024^2 float32, 32-node ER) configs
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for c in C5s C4; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/cfgprof_$c -o run --output-format csv -- \
    python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --strong none > gpurun_out/cfgprof_$c.log 2>&1 || exit $?
  python - "$c" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/cfgprof_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]:
    print(f'{sys.argv[1]} {float(r["AverageNs"])/1e3:9.2f} us x{int(r["Calls"]):4d} {float(r["Percentage"]):5.1f}%  {r["Name"][:70]}')
PY
done
