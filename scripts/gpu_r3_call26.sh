# Every -m gpu test after the chunk-aligned forward plan and float64 node-interleave 4,
# then the C4 / C5s config lines.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread --durations=8 > gpurun_out/pytest_r3b.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -14 gpurun_out/pytest_r3b.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/run_configs.sh C5s C4
