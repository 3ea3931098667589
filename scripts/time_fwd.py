"""Event-timed forward tap launches at the bench configuration (512^2, V=8), for one
library build (ADMM_TOMO_LIB): prints the average launch duration (diagnostic sweeps)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "distributed-inverse-problem-admm_amd"), ROOT]
import networkx as nx  # noqa: E402
import torch  # noqa: E402

from admm_hip.data import make_precisions, make_sinograms, shepp_logan  # noqa: E402
from admm_hip.plan import make_plan  # noqa: E402
from admm_hip.solver import NodeBatch, make_operators  # noqa: E402

V, N = int(os.environ.get("V", 8)), int(os.environ.get("N", 512))
ops = make_operators(N, V, angles_total=96 * V, device=0)
plan = make_plan(nx.cycle_graph(V), V, 1, 0)
ph = shepp_logan(N)
sinos = dict(zip(plan.local_nodes, make_sinograms(ops, ph, 0.005, seed=1000)))
Wi, Q = make_precisions(ops)
nb = NodeBatch(ops[0].geom, "float32", plan, sinos, Q, 2.0, 0.02, 0.2, 10, 5, "iso", ph, 0, keep_x=True)
nb.node_update()
torch.cuda.synchronize()
ts = [nb.time_forward(50) * 1e3 for _ in range(3)]
print(os.path.basename(os.environ.get("ADMM_TOMO_LIB", "default")), "fwd us/launch", [round(t, 2) for t in ts])
