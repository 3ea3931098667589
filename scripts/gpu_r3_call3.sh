set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize_projector.py tests/test_gpu_projector.py tests/test_gpu_admm.py tests/test_gpu_matrix.py -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/r3c3_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r3c3_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/probes/two_streams.py > gpurun_out/probe_2s.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/probe_2s.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 bash scripts/gpu_sweep.sh base kwin
