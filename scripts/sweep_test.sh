#!/bin/bash
# projector parity tests against each variants/*.so (ADMM_TOMO_LIB), then sweep_run.sh
set -u
mkdir -p gpurun_out
for so in variants/*.so; do
  ADMM_TOMO_LIB=$so timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize_projector.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pt_$(basename $so .so).log 2>&1
  rc=$?; echo "$so tests rc=$rc $(tail -1 gpurun_out/pt_$(basename $so .so).log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
bash scripts/sweep_run.sh && bash scripts/sweep_run.sh
