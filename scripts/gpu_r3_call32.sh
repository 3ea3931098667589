# Six forward plans (0-2 and their segment-clipped versions 3-5) and the picker: parity,
# bitwise plan equality, plan timings, bench lines vs the pre-clipping build, C4 / C5s.
set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_fullsize_projector.py tests/test_gpu_projector.py \
  tests/test_gpu_admm.py tests/test_gpu_matrix.py tests/test_gpu_bench.py "tests/test_gpu_configs.py::test_large_x_updates_match_operator_oracle" \
  -m gpu -q -x -rf --timeout 600 --timeout-method thread > gpurun_out/pytest_clip6.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_clip6.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u scripts/time_fwd_plans.py > gpurun_out/fwd_plans_clip.jsonl 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/fwd_plans_clip.jsonl
for i in 1 2; do
for v in new:distributed-inverse-problem-admm_amd/admm_hip/libadmm_tomo.so noclip:variants/lib_noclip.so; do
  name=${v%%:*}; lib=${v#*:}
  ADMM_TOMO_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --strong none > gpurun_out/ab_clip.json 2>/dev/null || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/ab_clip.json').read().strip().splitlines()[-1]); print('$name bench', round(d['value'],1), round(d['ms_per_step'],3), 'fwd', round(d['roofline']['avg_launch_ms']*1e3,2), d['roofline']['fwd_plan'])"
done
done
bash scripts/run_configs.sh C5s C4 C2 C3
