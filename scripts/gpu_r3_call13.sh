set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench.py tests/test_gpu_projector.py -m gpu -q -x -rf --timeout 200 --timeout-method thread > gpurun_out/r3c13_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r3c13_pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --strong none > gpurun_out/r3c13_bench$rep.json 2> gpurun_out/r3c13_bench$rep.err
  rc=$?; if [ $rc -ne 0 ]; then echo "bench rc=$rc"; tail -5 gpurun_out/r3c13_bench$rep.err; exit $rc; fi
  python -c "import json; b=json.load(open('gpurun_out/r3c13_bench$rep.json')); r=b['roofline']; print(round(b['value'],1), round(b['ms_per_step'],3), 'in-solve', round(r['avg_launch_ms']*1e3,2), 'b2b', round(r['avg_launch_ms_back_to_back']*1e3,2), 'frac', round(r['frac'],4))"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3c13 -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --strong none > gpurun_out/prof_r3c13.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
