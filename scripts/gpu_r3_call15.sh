# Fused back projector + CG update (BACK_HU, grid barrier) vs the three-launch form:
# solver parity and multi-rank bitwise tests on the in-tree (fused) library, bench lines of
# both variants, rocprofv3 kernel stats of both.
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_admm.py tests/test_gpu_multirank.py tests/test_gpu_dropins.py \
  -m gpu -q -x -rf --timeout 150 --timeout-method thread > gpurun_out/pytest_fuse.log 2>&1
rc=$?; echo "pytest fuse rc=$rc"; tail -4 gpurun_out/pytest_fuse.log
[ $rc -ne 0 ] && exit $rc
bash scripts/sweep_run.sh || exit $?
bash scripts/sweep_run.sh || exit $?
bash scripts/sweep_prof.sh
