# HBM traffic (PMC FETCH_SIZE / WRITE_SIZE, one pass each) of the C5s config line (2048^2,
# float64, plan 5), per kernel launch and per step (scripts/traffic_summary.py).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export ADMM_BENCH_MARKERS=1
i=0
for counters in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $counters --kernel-trace -d gpurun_out/c5pmc_$i -o run --output-format csv -- \
    python bench.py --config C5s --steps 1 --warmup 1 > gpurun_out/c5pmc_$i.log 2>&1
  rc=$?; echo "pass $i ($counters) rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/c5pmc_$i.log; exit $rc; }
done
python scripts/traffic_summary.py c5pmc 1 gpurun_out/c5s_traffic.json
