# A/B: clipped plans 3-5 grouped like their unclipped plans (variants/lib_keepg.so) -- the
# plans side by side at 512^2 / 1024^2 / 2048^2.
set -u
mkdir -p gpurun_out
ADMM_TOMO_LIB=variants/lib_keepg.so timeout -k 10 500 python -u scripts/time_fwd_plans.py > gpurun_out/fwd_plans_keepg.jsonl 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/fwd_plans_keepg.jsonl; exit $rc
