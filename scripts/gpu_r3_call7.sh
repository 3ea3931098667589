set -u
mkdir -p gpurun_out
ADMM_TOMO_LIB=variants/lib_wt.so timeout -k 10 400 python -u -m pytest tests/test_gpu_admm.py -m gpu -q -x -rf --timeout 200 --timeout-method thread > gpurun_out/r3c7_wt_pytest.log 2>&1
rc=$?; echo "wt pytest rc=$rc"; tail -2 gpurun_out/r3c7_wt_pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 bash scripts/gpu_sweep.sh base wt
