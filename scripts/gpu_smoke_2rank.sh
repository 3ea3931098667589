# smoke() + a 2-rank gloo rehearsal of the sharded bench on one GPU (the RCCL run is the driver's)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
ADMM_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --strong C4 > gpurun_out/bench_2rank_gloo.json 2> gpurun_out/bench_2rank_gloo.err
rc=$?; echo "2-rank rc=$rc"; cat gpurun_out/bench_2rank_gloo.json | cut -c1-300; tail -3 gpurun_out/bench_2rank_gloo.err
exit $rc
