set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/probes/vb_bitwise.py > gpurun_out/probe_vb2.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/probe_vb2.log | tail -12; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --strong none > gpurun_out/r3c2_bench.json 2> gpurun_out/r3c2_bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/r3c2_bench.json
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 1000 python -u -m pytest tests -m gpu --ignore=tests/test_gpu_configs_full.py -v -x -rf --timeout 400 --timeout-method thread > gpurun_out/r3c2_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r3c2_pytest.log
true
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 bash scripts/gpu_sweep.sh base bk16
