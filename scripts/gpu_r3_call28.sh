# Back projector H mode with the tile's r rows prefetched into LDS by LDS-DMA: projector and
# ADMM parity, then rocprofv3 kernel stats + bench lines vs the previous build (lib_norpf).
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_projector.py tests/test_gpu_admm.py tests/test_gpu_dropins.py \
  -m gpu -q -x -rf --timeout 200 --timeout-method thread > gpurun_out/pytest_rpf.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_rpf.log
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
for v in rpf:distributed-inverse-problem-admm_amd/admm_hip/libadmm_tomo.so norpf:variants/lib_norpf.so; do
  name=${v%%:*}; lib=${v#*:}
  ADMM_TOMO_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --strong none > gpurun_out/ab_rpf.json 2>/dev/null || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/ab_rpf.json').read().strip().splitlines()[-1]); print('$name bench', round(d['value'],1), round(d['ms_per_step'],3))"
done
done
for v in rpf:distributed-inverse-problem-admm_amd/admm_hip/libadmm_tomo.so norpf:variants/lib_norpf.so; do
  name=${v%%:*}; lib=${v#*:}
  ADMM_TOMO_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o run --output-format csv -- \
    python bench.py --steps 10 --warmup 3 --no-cpu-baseline --strong none > gpurun_out/prof_$name.log 2>&1 || exit $?
  echo "== $name"; python scripts/top_kernels.py gpurun_out/prof_$name | head -6
done
