set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/probes/step_sync.py > gpurun_out/probe_sync.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/probe_sync.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 1000 python -u -m pytest tests/test_gpu_configs_full.py -m gpu -v -x -rf -s --timeout 900 --timeout-method thread > gpurun_out/r3c4_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|C4 graph|'x'|passed|failed" gpurun_out/r3c4_pytest.log | tail -12
exit $rc
