"""Probe: the 8-node x-update as ONE batch (VB=8) vs TWO 4-node batches (VB=4) replayed on two
streams concurrently (their kernels overlap each other's dependent-launch boundaries)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "distributed-inverse-problem-admm_amd"), ROOT]
import networkx as nx  # noqa: E402
import torch  # noqa: E402
from admm_hip.data import make_precisions, make_sinograms, shepp_logan  # noqa: E402
from admm_hip.plan import make_plan, make_subset_plan  # noqa: E402
from admm_hip.solver import NodeBatch, make_operators  # noqa: E402

N, V = 512, 8
ops = make_operators(N, V, 96 * V, device=0)
ph = shepp_logan(N)
sinos = make_sinograms(ops, ph, 0.005, seed=1000)
Wi, Q = make_precisions(ops)
G = nx.cycle_graph(V)
geom = ops[0].geom


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


one = NodeBatch(geom, "float32", make_plan(G, V), sinos, Q, 2.0, 0.02, 0.2, 10, 5, "iso", ph, 0, keep_x=True)
print(f"one batch of 8 (VB=8): {timeit(one.node_update):.3f} ms per x-update of 8 nodes")
del one
halves = [NodeBatch(geom, "float32", make_subset_plan(G, V, range(h * 4, h * 4 + 4)), sinos, Q, 2.0, 0.02, 0.2,
                    10, 5, "iso", ph, 0, keep_x=True) for h in range(2)]
streams = [torch.cuda.Stream() for _ in range(2)]


def serial():
    for nb in halves:
        nb.node_update()


def concurrent():
    cur = torch.cuda.current_stream()
    for nb, s in zip(halves, streams):
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            nb.node_update()
    for s in streams:
        cur.wait_stream(s)


print(f"two batches of 4 (VB=4), one stream: {timeit(serial):.3f} ms")
print(f"two batches of 4 (VB=4), two streams: {timeit(concurrent):.3f} ms")
