#!/bin/bash
# BASELINE.json configs on one GPU (bench.py --config); one JSON line each
set -u
mkdir -p gpurun_out
for c in "$@"; do
  timeout -k 10 900 python bench.py --config $c --steps 3 --warmup 1 > gpurun_out/config_$c.json 2> gpurun_out/config_$c.err
  rc=$?
  echo "$c rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/config_$c.err; exit $rc; fi
  python -c "import json; b=json.load(open('gpurun_out/config_$c.json')); print('$c', round(b['value'],2), 'node-updates/s', round(b['ms_per_step'],1), 'ms/step', 'fwd', round(b['roofline']['avg_launch_ms']*1e3,1), 'us')"
done
