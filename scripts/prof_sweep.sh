#!/bin/bash
# rocprofv3 kernel stats of bench.py for each variants/*.so (kernel-trace only)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for so in variants/*.so; do
  tag=$(basename $so .so)
  ADMM_TOMO_LIB=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/vprof_$tag -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/vprof_$tag.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$so rc=$rc"; exit $rc; fi
  echo "$so ok"
done
