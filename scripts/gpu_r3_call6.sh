set -u
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/test_gpu_configs_full.py -m gpu -v -x -rf -s --timeout 900 --timeout-method thread --durations=5 > gpurun_out/r3c6_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|C4 graph|'x'|passed|failed|s call" gpurun_out/r3c6_pytest.log | tail -14
exit $rc
