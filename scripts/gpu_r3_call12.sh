set -u
mkdir -p gpurun_out
ADMM_TOMO_LIB=variants/lib_f64dma.so timeout -k 10 500 python -u -m pytest tests/test_gpu_admm.py tests/test_gpu_projector.py tests/test_gpu_fullsize_projector.py -m gpu -q -x -rf --timeout 200 --timeout-method thread > gpurun_out/r3c12_f64dma_pytest.log 2>&1
rc=$?; echo "f64dma pytest rc=$rc"; tail -2 gpurun_out/r3c12_f64dma_pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
for v in base f64dma base f64dma; do
  ADMM_TOMO_LIB=variants/lib_$v.so timeout -k 10 300 python bench.py --config C5s --steps 4 --warmup 1 --no-cpu-baseline --strong none > gpurun_out/c5s_$v.json 2> gpurun_out/c5s_$v.err
  rc=$?; if [ $rc -ne 0 ]; then echo "$v rc=$rc"; tail -5 gpurun_out/c5s_$v.err; exit $rc; fi
  python -c "import json; b=json.load(open('gpurun_out/c5s_$v.json')); print('$v', round(b['value'],2), round(b['ms_per_step'],2), round(b['roofline']['avg_launch_ms']*1e3,1))"
done
