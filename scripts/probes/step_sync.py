"""Probe: what the per-step statistics read-back (a host sync every ADMM iteration) costs the
bench step: (a) as bench.py runs it, (b) read-back copied asynchronously into pinned host
memory (no per-step sync), (c) no read-back at all (upper bound)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "distributed-inverse-problem-admm_amd"), ROOT]
import torch  # noqa: E402
import bench  # noqa: E402
from admm_hip.exchange import assemble_stats  # noqa: E402

torch.cuda.set_device(0)
r = bench.setup_run("weak8", 1, 0, 0)
nb, halo, plan = r["nb"], r["rg"].halo, r["plan"]
E = len(plan.stored_edges)
hs = torch.empty(nb.node_stats.shape, dtype=torch.float64, pin_memory=True)
he = torch.empty((max(E, 1), nb.edge_stats.shape[1]), dtype=torch.float64, pin_memory=True)


def sync_step():
    nb.node_update(); halo.run(); nb.consensus()
    return assemble_stats(plan, nb.node_stats, nb.edge_stats[:E])


def async_step():
    nb.node_update(); halo.run(); nb.consensus()
    hs.copy_(nb.node_stats, non_blocking=True)
    he.copy_(nb.edge_stats[: max(E, 1)], non_blocking=True)


def bare_step():
    nb.node_update(); halo.run(); nb.consensus()


for name, fn in (("sync", sync_step), ("async", async_step), ("none", bare_step)) * 2:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(30):
        fn()
    torch.cuda.synchronize()
    print(f"{name:6s} {1e3 * (time.perf_counter() - t) / 30:.4f} ms/step")
