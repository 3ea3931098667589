#!/bin/bash
# One GPU session: parity tests, short bench, rocprofv3 kernel stats.
# Stops at the first crash / timeout (exit codes other than 0/1 from pytest).
set -u
mkdir -p gpurun_out
TAG=${1:-r2}
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rA --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -5 gpurun_out/bench_$TAG.err
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
rc=$?
echo "rocprof rc=$rc"
find gpurun_out/prof_$TAG -name "*stats*"
exit $rc
