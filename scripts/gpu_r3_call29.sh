# Bench-line checks (plan field, certificate objective) and the default bench line with the CPU baseline.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench.py -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_bench.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_bench.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r3c.json 2> gpurun_out/bench_r3c.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_r3c.json; exit $rc
