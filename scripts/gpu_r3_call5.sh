set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/probes/multirank_bisect.py > gpurun_out/bisect_fixed.log 2>&1
rc=$?; grep -v "amdgpu.ids\|Gloo\|socket.cpp\|primal" gpurun_out/bisect_fixed.log | tail -6; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 700 python -u -m pytest tests/test_gpu_admm.py tests/test_gpu_multirank.py tests/test_gpu_groups.py tests/test_gpu_bench.py tests/test_gpu_matrix.py tests/test_gpu_configs.py -m gpu -q -x -rf --timeout 400 --timeout-method thread > gpurun_out/r3c5_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r3c5_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --strong none > gpurun_out/r3c5_bench$rep.json 2> gpurun_out/r3c5_bench$rep.err
rc=$?; echo "bench rc=$rc"; python -c "import json; b=json.load(open('gpurun_out/r3c5_bench$rep.json')); print(round(b['value'],1), round(b['ms_per_step'],4), round(b['roofline']['avg_launch_ms']*1e3,2))"
if [ $rc -ne 0 ]; then exit $rc; fi
done
