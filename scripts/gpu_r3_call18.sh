# Diagnostic (not a product variant): forward projector with the in-loop barriers not waiting
# for the LDS-DMA (taps may read stale rows; timing only) vs the product kernel.
set -u
mkdir -p gpurun_out
bash scripts/sweep_run.sh || exit $?
bash scripts/sweep_run.sh || exit $?
bash scripts/sweep_prof.sh
