# Full GPU check of the in-tree library: HBM traffic passes (first: the bench line the
# tests check reads them), every -m gpu test,
# kernel-trace stats and the default bench line (with the CPU baseline).  usage: gpu_full_check.sh TAG
set -u
mkdir -p gpurun_out
TAG=${1:-r3}
bash scripts/pmc.sh $TAG > gpurun_out/pmc_$TAG.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -4 gpurun_out/pmc_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
cp gpurun_out/${TAG}_traffic.json profiles/${TAG}_traffic.json
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 200 --timeout-method thread --durations=10 > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -14 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --headline-only > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke_$TAG.log
exit $rc
