set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_matrix.py tests/test_gpu_projector.py tests/test_gpu_admm.py tests/test_gpu_dropins.py -m gpu -v -x --timeout 200 --timeout-method thread > gpurun_out/pt_g6.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pt_g6.log | tail -12
exit $rc
