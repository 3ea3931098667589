"""Host time of the per-iteration launches of the C3 bench workload (no synchronisation between
iterations): if a graph launch blocked until the previous launch of the same exec finished, each
node_update() call would cost about a whole GPU step on the host.  Measured (round 5): 0.07 ms
per graph launch, 0.7 ms enqueued directly -- the host stays ahead (AB_LOG).  The printed
"PINGPONG" tag is the ADMM_GRAPH_PINGPONG value of that A/B (the switch itself was removed)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import bench  # noqa: E402
import torch  # noqa: E402

r = bench.setup_run("C3", 1, 0, 0)
rg = r["rg"]
for _ in range(3):
    rg.node_update()
    rg.exchange_consensus()
torch.cuda.synchronize()
t_upd, t_con, t_all = [], [], time.perf_counter()
for _ in range(20):
    a = time.perf_counter()
    rg.node_update()
    b = time.perf_counter()
    rg.exchange_consensus()
    c = time.perf_counter()
    t_upd.append(b - a)
    t_con.append(c - b)
torch.cuda.synchronize()
t_all = time.perf_counter() - t_all
print(f"PINGPONG={os.environ.get('ADMM_GRAPH_PINGPONG', '0')}: node_update host ms "
      f"{[round(1e3 * x, 2) for x in t_upd[:8]]} ... consensus host ms {[round(1e3 * x, 3) for x in t_con[:4]]}; "
      f"20 iterations {1e3 * t_all / 20:.3f} ms each")
