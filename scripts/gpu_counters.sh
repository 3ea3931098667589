# Profile the default bench: HBM traffic passes, SQ counter passes, kernel-trace stats.
set -u
mkdir -p gpurun_out
TAG=${1:-r2b}
bash scripts/pmc.sh $TAG > gpurun_out/pmc_$TAG.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -30 gpurun_out/pmc_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
PASSFILE=scripts/pmc_sq2.txt bash scripts/pmc.sh ${TAG}sq > gpurun_out/pmc_${TAG}sq.log 2>&1
rc=$?; echo "pmc sq rc=$rc"; tail -5 gpurun_out/pmc_${TAG}sq.log
if [ $rc -ne 0 ]; then exit $rc; fi
python scripts/pmc_summary.py ${TAG}sq > gpurun_out/${TAG}_sq_summary.txt 2>&1; tail -40 gpurun_out/${TAG}_sq_summary.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --strong none > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof_$TAG.log
exit $rc
