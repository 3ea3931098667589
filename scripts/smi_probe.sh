#!/bin/bash
# power / clock readings idle and under the C3 bench (read-only rocm-smi queries)
mkdir -p gpurun_out
timeout -k 5 30 rocm-smi --showmaxpower --showpower --showclocks --showtemp > gpurun_out/smi_idle.txt 2>&1
timeout -k 10 200 python bench.py --steps 3000 --warmup 5 --no-cpu-baseline --headline-only > gpurun_out/smi_bench.json 2> gpurun_out/smi_bench.err &
BP=$!
for k in 1 2 3 4 5 6; do
  sleep 5
  timeout -k 5 20 rocm-smi --showpower --showclocks --showtemp > gpurun_out/smi_load_$k.txt 2>&1
done
wait $BP
echo "bench rc=$?"
