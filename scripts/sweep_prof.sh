#!/bin/bash
# rocprofv3 kernel stats of bench.py for each variants/*.so (per-kernel average durations)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for so in variants/*.so; do
  tag=$(basename $so .so)
  ADMM_TOMO_LIB=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sp_$tag -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --strong none > gpurun_out/sp_$tag.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "$so rc=$rc"; tail -5 gpurun_out/sp_$tag.log; exit $rc; fi
  echo "== $tag $(grep -o '"value": [0-9.]*' gpurun_out/sp_$tag.log)"
  python - "$tag" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/sp_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:9]:
    print(f'  {float(r["AverageNs"])/1e3:8.2f} us x{int(r["Calls"]):4d} {float(r["Percentage"]):5.1f}%  {r["Name"][:60]}')
PY
done
