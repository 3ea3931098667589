# A/B of variants/*.so: bench value + forward launch time per variant, then rocprofv3 kernel stats
# usage: gpu_sweep.sh NAME [NAME ...]   (variants/lib_NAME.so built by sweep_build.py)
set -u
mkdir -p gpurun_out
for v in "$@"; do
  for rep in 1 2; do
    ADMM_TOMO_LIB=variants/lib_$v.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --strong none > gpurun_out/sweep_${v}_$rep.json 2> gpurun_out/sweep_${v}_$rep.err
    rc=$?; if [ $rc -ne 0 ]; then echo "$v rc=$rc"; tail -5 gpurun_out/sweep_${v}_$rep.err; exit $rc; fi
    python -c "import json; b=json.load(open('gpurun_out/sweep_${v}_$rep.json')); print('$v', $rep, round(b['value'],1), round(b['ms_per_step'],3), round(b['roofline']['avg_launch_ms']*1e3,2))"
  done
done
bash scripts/prof_variants.sh "$@"
