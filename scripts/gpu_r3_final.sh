# Final state: every -m gpu test and the smoke check.
set -u
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 600 --timeout-method thread > gpurun_out/pytest_final.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_final.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_final.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke_final.log; exit $rc
