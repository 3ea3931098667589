"""Does the event-timed forward launch depend on the repetition count?  (measurement check)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-inverse-problem-admm_amd"))
sys.path.insert(0, ROOT)
import networkx as nx  # noqa: E402
import torch  # noqa: E402

from admm_hip.data import make_precisions, make_sinograms, shepp_logan  # noqa: E402
from admm_hip.plan import make_plan  # noqa: E402
from admm_hip.solver import NodeBatch, make_operators  # noqa: E402

torch.cuda.set_device(0)
V, N = 8, 512
ops = make_operators(N, V, angles_total=96 * V, device=0)
G = nx.cycle_graph(V)
plan = make_plan(G, V, 1, 0)
ph = shepp_logan(N)
sinos = dict(zip(plan.local_nodes, make_sinograms(ops, ph, 0.005, seed=1000)))
Wi, Q = make_precisions(ops)
nb = NodeBatch(ops[0].geom, "float32", plan, sinos, Q, 2.0, 0.02, 0.2, 10, 5, "iso", ph, 0, keep_x=True)
nb.node_update()
torch.cuda.synchronize()
for reps in (1, 2, 5, 20, 100, 20, 1):
    print(reps, round(nb.time_forward(reps) * 1e3, 2), "us/launch", flush=True)
