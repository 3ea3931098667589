# 8-rank rehearsals on one GPU (gloo): bench --gpus 8 with the C4 strong leg, C4 over 4 / 8
# ranks bitwise, and the multirank suite.
set -u
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_bench.py tests/test_gpu_multirank.py \
  "tests/test_gpu_configs_full.py::test_c4_ranks_match_one_rank_bitwise" -m gpu -v -x -rf \
  --timeout 900 --timeout-method thread --durations=6 > gpurun_out/pytest_8rank.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E 'PASS|FAIL|ERROR|passed|failed' gpurun_out/pytest_8rank.log | tail -25
exit $rc
