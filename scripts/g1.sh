set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize_projector.py tests/test_gpu_projector.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pt_g1.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pt_g1.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/pmc.sh r2a > gpurun_out/pmc_r2a.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -30 gpurun_out/pmc_r2a.log
if [ $rc -ne 0 ]; then exit $rc; fi
cp gpurun_out/r2a_traffic.json profiles/r2_traffic.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_g1.json 2> gpurun_out/bench_g1.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_g1.json; tail -5 gpurun_out/bench_g1.err
exit $rc
