set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_groups.py tests/test_gpu_multirank.py tests/test_gpu_bench.py tests/test_gpu_dropins.py tests/test_gpu_matrix.py tests/test_gpu_admm.py -m gpu -v -x -rf --timeout 300 --timeout-method thread > gpurun_out/r3c1_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/r3c1_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --strong none > gpurun_out/r3c1_bench.json 2> gpurun_out/r3c1_bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/r3c1_bench.json
exit $rc
