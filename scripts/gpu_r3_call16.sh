# Forward projector: one LDS-DMA buffer of 8 or 16 rows per chunk (stage, barrier, taps, barrier)
# and 8-row double buffers vs the 2-row double buffer: projector parity on the 8-row single
# buffer, bench lines and rocprofv3 kernel stats of each variant.
set -u
mkdir -p gpurun_out
ADMM_TOMO_LIB=variants/lib_r8n1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_projector.py \
  tests/test_gpu_fullsize_projector.py -m gpu -q -x -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_r8n1.log 2>&1
rc=$?; echo "pytest r8n1 rc=$rc"; tail -3 gpurun_out/pytest_r8n1.log
[ $rc -ne 0 ] && exit $rc
bash scripts/sweep_run.sh || exit $?
bash scripts/sweep_run.sh || exit $?
bash scripts/sweep_prof.sh
