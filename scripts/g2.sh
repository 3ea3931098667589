set -u
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/test_gpu_dropins.py tests/test_gpu_configs.py tests/test_gpu_admm.py tests/test_gpu_fullsize.py tests/test_gpu_multirank.py -m gpu -v -rA --timeout 150 --timeout-method thread --durations=15 > gpurun_out/pt_g2.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|slowest" gpurun_out/pt_g2.log | tail -45
exit $rc
