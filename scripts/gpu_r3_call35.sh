# After shrinking FgGroup to (t0, G): projector / ADMM / plan-bitwise / matrix / bench tests and a bench line.
set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_fullsize_projector.py tests/test_gpu_projector.py \
  tests/test_gpu_admm.py tests/test_gpu_matrix.py tests/test_gpu_bench.py -m gpu -q -x -rf --timeout 600 \
  --timeout-method thread > gpurun_out/pytest_fggroup.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_fggroup.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --strong none > gpurun_out/b.json 2>/dev/null || exit $?
python -c "import json; d=json.loads(open('gpurun_out/b.json').read().strip().splitlines()[-1]); print('bench', round(d['value'],1), round(d['ms_per_step'],3), 'fwd', round(d['roofline']['avg_launch_ms']*1e3,2), d['roofline']['fwd_plan']['plan'])"
