set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/probes/vb_bitwise.py > gpurun_out/probe_vb.log 2>&1
rc=$?; cat gpurun_out/probe_vb.log | grep -v amdgpu.ids; exit $rc
