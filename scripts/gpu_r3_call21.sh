# Chunk-aligned forward plan (2): projector parity on every plan, bitwise plan equality of
# whole ADMM runs, then the plans side by side (planner stats + event-timed tap launches).
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize_projector.py tests/test_gpu_projector.py \
  "tests/test_gpu_admm.py::test_forward_plans_bitwise_equal" -m gpu -q -x -rf --timeout 200 \
  --timeout-method thread > gpurun_out/pytest_plan2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_plan2.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/time_fwd_plans.py > gpurun_out/fwd_plans.jsonl 2>&1
rc=$?; cat gpurun_out/fwd_plans.jsonl; exit $rc
