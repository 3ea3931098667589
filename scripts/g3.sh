set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize_projector.py tests/test_gpu_projector.py tests/test_gpu_admm.py -m gpu -q -x --timeout 150 --timeout-method thread > gpurun_out/pt_g3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_g3.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/sweep_run.sh && bash scripts/sweep_run.sh
