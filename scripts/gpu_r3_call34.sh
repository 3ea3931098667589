# A/B: float64 back projector window prefetch (PF) on / off at C5s (node interleave 4).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in pf64 nopf64; do
  ADMM_TOMO_LIB=variants/lib_$v.so timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5s_$v -o run --output-format csv -- \
    python bench.py --config C5s --steps 3 --warmup 1 > gpurun_out/c5s_$v.json 2> gpurun_out/c5s_$v.err || exit $?
  python -c "import json; b=json.load(open('gpurun_out/c5s_$v.json')); print('$v C5s', round(b['value'],2), round(b['ms_per_step'],1))"
  python scripts/top_kernels.py gpurun_out/prof_c5s_$v | head -3
done
