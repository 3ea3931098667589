#!/bin/bash
# time bench.py against each variants/*.so (ADMM_TOMO_LIB); one line per variant
set -u
mkdir -p gpurun_out
for so in variants/*.so; do
  ADMM_TOMO_LIB=$so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/sweep_$(basename $so .so).json 2>/dev/null
  rc=$?
  if [ $rc -ne 0 ]; then echo "$so rc=$rc"; exit $rc; fi
  python -c "import json,sys; b=json.load(open('gpurun_out/sweep_$(basename $so .so).json')); print('$so', round(b['value'],1), round(b['roofline']['avg_launch_ms']*1e3,2))"
done
