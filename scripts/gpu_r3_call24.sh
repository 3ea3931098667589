# rocprofv3 kernel stats of the C5s config line, float64 node-interleave 8 (default) vs 4.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in vb8:distributed-inverse-problem-admm_amd/admm_hip/libadmm_tomo.so vb4:variants/lib_f64vb4.so; do
  name=${v%%:*}; lib=${v#*:}
  ADMM_TOMO_LIB=$lib timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5s_$name -o run --output-format csv -- \
    python bench.py --config C5s --steps 3 --warmup 1 > gpurun_out/c5s_$name.json 2> gpurun_out/c5s_$name.err || exit $?
  f=$(find gpurun_out/prof_c5s_$name -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/c5s_${name}_kernel_stats.csv
  python scripts/top_kernels.py gpurun_out/prof_c5s_$name > gpurun_out/c5s_${name}_top.txt; cat gpurun_out/c5s_${name}_top.txt
done
