# Quick A/B of the in-tree library: projector + ADMM parity tests, rocprofv3 kernel stats of
# the default bench, one bench line.  usage: gpu_quick.sh TAG
set -u
mkdir -p gpurun_out
TAG=${1:-quick}
timeout -k 10 400 python -u -m pytest tests/test_gpu_projector.py tests/test_gpu_fullsize_projector.py \
  tests/test_gpu_admm.py -m gpu -q -x -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --strong none > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
python scripts/top_kernels.py gpurun_out/prof_$TAG
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --strong none > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 gpurun_out/bench_$TAG.json
exit $rc
