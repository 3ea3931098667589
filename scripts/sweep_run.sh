#!/bin/bash
# time bench.py against each variants/*.so (ADMM_TOMO_LIB), optionally under extra env settings
# usage: sweep_run.sh ["ENV=VAL ENV2=VAL" ...]   (each argument = one env setting; default: none)
set -u
mkdir -p gpurun_out
settings=("$@")
[ ${#settings[@]} -eq 0 ] && settings=("")
for so in variants/*.so; do
  for st in "${settings[@]}"; do
    tag=$(basename $so .so)_$(echo "$st" | tr ' =' '__')
    env $st ADMM_TOMO_LIB=$so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --strong none > gpurun_out/sweep_$tag.json 2>/dev/null
    rc=$?
    if [ $rc -ne 0 ]; then echo "$so [$st] rc=$rc"; exit $rc; fi
    python -c "import json; b=json.load(open('gpurun_out/sweep_$tag.json')); print('$so', '[$st]', round(b['value'],1), round(b['roofline']['avg_launch_ms']*1e3,2))"
  done
done
