# Forward projector with two angle slots per wave (ADMM_FG_APW=2) vs one, and the HEAD build:
# parity tests on the APW=2 library, bench lines and rocprofv3 kernel stats of each variant.
set -u
mkdir -p gpurun_out
ADMM_TOMO_LIB=variants/lib_apw2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_projector.py \
  tests/test_gpu_fullsize_projector.py tests/test_gpu_admm.py -m gpu -q -x -rf --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_apw2.log 2>&1
rc=$?; echo "pytest apw2 rc=$rc"; tail -3 gpurun_out/pytest_apw2.log
[ $rc -ne 0 ] && exit $rc
bash scripts/sweep_run.sh || exit $?
bash scripts/sweep_run.sh || exit $?
bash scripts/sweep_prof.sh
