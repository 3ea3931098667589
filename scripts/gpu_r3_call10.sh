set -u
mkdir -p gpurun_out
for v in g12w320; do
  ADMM_TOMO_LIB=variants/lib_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_admm.py tests/test_gpu_projector.py tests/test_gpu_fullsize_projector.py -m gpu -q -x -rf --timeout 200 --timeout-method thread > gpurun_out/r3c10_${v}_pytest.log 2>&1
  rc=$?; echo "$v pytest rc=$rc"; tail -2 gpurun_out/r3c10_${v}_pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 900 bash scripts/gpu_sweep.sh base g12w320
