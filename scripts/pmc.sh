#!/bin/bash
# PMC passes (each its own run, kernel-trace only, per MI355X_MICROARCH.md guidance)
set -u
mkdir -p gpurun_out
TAG=${1:-pmc}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
CMD="python bench.py --steps 2 --warmup 1 --no-cpu-baseline"
i=0
if [ -n "${PASSFILE:-}" ]; then mapfile -t PASSLIST < "$PASSFILE"; else PASSLIST=("FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"); fi
for counters in "${PASSLIST[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $counters --kernel-trace -d gpurun_out/${TAG}_$i -o run --output-format csv -- $CMD > gpurun_out/${TAG}_$i.log 2>&1
  rc=$?
  echo "pass $i ($counters) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_$i.log; exit $rc; fi
done
