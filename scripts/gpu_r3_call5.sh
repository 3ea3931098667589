set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_admm.py tests/test_gpu_multirank.py tests/test_gpu_groups.py tests/test_gpu_bench.py tests/test_gpu_matrix.py -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/r3c5_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r3c5_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --strong none > gpurun_out/r3c5_bench$rep.json 2> gpurun_out/r3c5_bench$rep.err
rc=$?; echo "bench rc=$rc"; python -c "import json; b=json.load(open('gpurun_out/r3c5_bench$rep.json')); print(round(b['value'],1), round(b['ms_per_step'],4), round(b['roofline']['avg_launch_ms']*1e3,2))"
if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 1000 python -u -m pytest "tests/test_gpu_configs_full.py::test_c5_full_graph_one_gpu_and_two_ranks" -m gpu -v -x -rf -s --timeout 900 --timeout-method thread > gpurun_out/r3c5_c5.log 2>&1
rc=$?; echo "c5 rc=$rc"; grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/r3c5_c5.log | tail -5
exit $rc
