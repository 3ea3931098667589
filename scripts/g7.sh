set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_admm.py tests/test_gpu_configs.py tests/test_gpu_multirank.py tests/test_gpu_dropins.py tests/test_gpu_fullsize.py tests/test_gpu_matrix.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pt_g7.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_g7.log
[ $rc -ne 0 ] && exit $rc
bash scripts/sweep_run.sh && bash scripts/sweep_run.sh
