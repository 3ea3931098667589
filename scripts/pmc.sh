#!/bin/bash
# HBM traffic passes (FETCH_SIZE, WRITE_SIZE: each its own run, kernel-trace only, per
# MI355X_MICROARCH.md) over the default bench workload with marker kernels around the
# timed steps; then scripts/traffic_summary.py.  usage: scripts/pmc.sh TAG
set -u
mkdir -p gpurun_out
TAG=${1:-pmc}
STEPS=2
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export ADMM_BENCH_MARKERS=1
i=0
if [ -n "${PASSFILE:-}" ]; then mapfile -t PASSLIST < "$PASSFILE"; else PASSLIST=("FETCH_SIZE" "WRITE_SIZE"); fi
for counters in "${PASSLIST[@]}"; do
  i=$((i+1))
  timeout -s KILL ${PASS_TIMEOUT:-300} rocprofv3 --pmc $counters --kernel-trace -d gpurun_out/${TAG}_$i -o run --output-format csv -- python bench.py --steps $STEPS --warmup 1 --no-cpu-baseline --headline-only --workload ${WORKLOAD:-C3} > gpurun_out/${TAG}_$i.log 2>&1
  rc=$?
  echo "pass $i ($counters) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_$i.log; exit $rc; fi
done
if [ -z "${PASSFILE:-}" ]; then python scripts/traffic_summary.py $TAG $STEPS gpurun_out/${TAG}_traffic.json; fi
