# float64 x 8 forward as two 2-plane halves (split blocks): projector / ADMM parity, then
# rocprofv3 kernel stats of C5s for the default build and the node-interleave-4 variant.
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize_projector.py tests/test_gpu_projector.py \
  tests/test_gpu_admm.py -m gpu -q -x -rf --timeout 200 --timeout-method thread > gpurun_out/pytest_split.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_split.log
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in split:distributed-inverse-problem-admm_amd/admm_hip/libadmm_tomo.so vb4:variants/lib_f64vb4.so; do
  name=${v%%:*}; lib=${v#*:}
  ADMM_TOMO_LIB=$lib timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5s_$name -o run --output-format csv -- \
    python bench.py --config C5s --steps 3 --warmup 1 > gpurun_out/c5s_$name.json 2> gpurun_out/c5s_$name.err || exit $?
  python -c "import json; b=json.load(open('gpurun_out/c5s_$name.json')); print('$name C5s', round(b['value'],2), 'node-updates/s', round(b['ms_per_step'],1), 'ms/step')"
  python scripts/top_kernels.py gpurun_out/prof_c5s_$name | head -6
done
