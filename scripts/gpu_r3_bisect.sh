set -u
mkdir -p gpurun_out
for m in sync_exchange sync_stats sync_update; do
PROBE_MODE=$m ADMM_TOMO_LIB=variants/lib_cur.so timeout -k 10 300 python -u scripts/probes/multirank_bisect.py > gpurun_out/bisect_$m.log 2>&1
rc=$?; grep -v "amdgpu.ids\|Gloo\|socket.cpp" gpurun_out/bisect_$m.log | tail -8; if [ $rc -ne 0 ]; then exit $rc; fi
done
