# Forward projector: 3-buffer LDS-DMA ring (inline-asm DMA, counted vmcnt, the chunk after next
# in flight across each barrier) vs the 2-buffer product kernel: projector + solver parity on
# the ring, bench lines, rocprofv3 kernel stats.
set -u
mkdir -p gpurun_out
ADMM_TOMO_LIB=variants/lib_ring3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_projector.py \
  tests/test_gpu_fullsize_projector.py tests/test_gpu_admm.py -m gpu -q -x -rf --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_ring3.log 2>&1
rc=$?; echo "pytest ring3 rc=$rc"; tail -3 gpurun_out/pytest_ring3.log
[ $rc -ne 0 ] && exit $rc
bash scripts/sweep_run.sh || exit $?
bash scripts/sweep_run.sh || exit $?
bash scripts/sweep_prof.sh
