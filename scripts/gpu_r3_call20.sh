# Forward segment partials stored write-through (sc1) and a MODE-0 combine with 2 threads per ray,
# alone and together, vs the product kernels: solver parity on the combined variant, bench lines,
# rocprofv3 kernel stats.
set -u
mkdir -p gpurun_out
ADMM_TOMO_LIB=variants/lib_wtsplit2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_projector.py \
  tests/test_gpu_admm.py -m gpu -q -x -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_wtsplit2.log 2>&1
rc=$?; echo "pytest wtsplit2 rc=$rc"; tail -3 gpurun_out/pytest_wtsplit2.log
[ $rc -ne 0 ] && exit $rc
bash scripts/sweep_run.sh || exit $?
bash scripts/sweep_run.sh || exit $?
bash scripts/sweep_prof.sh
