"""Probe: is the forward projector's output for one image bitwise independent of how many
images share the launch (VB = 1, 2, 4, 8)?  Prints max |diff| of image 0 vs the VB=8 launch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "distributed-inverse-problem-admm_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from admm_hip.geometry import ParallelBeamGeometry, RayTransform  # noqa: E402

for N, a in ((40, 17), (40, 16), (512, 96)):
    op = RayTransform(ParallelBeamGeometry(N, a), "float32", 0)
    rng = np.random.default_rng(0)
    X = torch.as_tensor(rng.standard_normal((8, N * N)), dtype=torch.float32, device="cuda")
    ref = (op @ X)[0].cpu().numpy()
    refT = (op.T @ (op @ X))[0].cpu().numpy()
    for k in (1, 2, 3, 4, 5, 8):
        y = (op @ X[:k])[0].cpu().numpy()
        print(f"N={N} a={a} k={k}: fwd max|d|={np.abs(y - ref).max():.3e} equal={np.array_equal(y, ref)}")
    for plan in ("0", "1"):
        os.environ["ADMM_FWD_PLAN"] = plan
        y = (RayTransform(ParallelBeamGeometry(N, a), "float32", 0) @ X[:1])[0].cpu().numpy()
        print(f"  plan {plan}: equal={np.array_equal(y, ref)}")
    os.environ.pop("ADMM_FWD_PLAN", None)

# the batch path: node 0's x-update alone (V=1, VB=1) and inside batches of V = 2, 3, 4, 8
import networkx as nx  # noqa: E402
from admm_hip.data import make_precisions, make_sinograms, shepp_logan  # noqa: E402
from admm_hip.plan import make_plan  # noqa: E402
from admm_hip.solver import NodeBatch, make_operators  # noqa: E402
N = 40
ops = make_operators(N, 8, 8 * 17, device=0)
ph = shepp_logan(N)
sinos = make_sinograms(ops, ph, 0.005, seed=1000)
sinos = [sinos[0]] * 8
Wi, Q = make_precisions(ops)
res = {}
for V in (1, 2, 3, 4, 8):
    G = nx.empty_graph(V)
    nb = NodeBatch(ops[0].geom, "float32", make_plan(G, V), sinos, Q, 2.0, 0.02, 0.2, 10, 5, "iso", ph, 0)
    for _ in range(2):
        nb.node_update()
    res[V] = (nb.x_local[0].cpu().numpy().copy(), nb.node_stats[0].cpu().numpy().copy())
    print(f"batch V={V}: x equal to V=1: {np.array_equal(res[V][0], res[1][0])} "
          f"max|d|={np.abs(res[V][0] - res[1][0]).max():.3e}  stats equal: {np.array_equal(res[V][1], res[1][1])}")

# with edges: node 0 of a 6-node complete graph in batches {0}, {0,1}, {0,1,2}, {0..3};
# halo rows / edge state filled with the same fixed random data
from admm_hip.plan import make_subset_plan  # noqa: E402
G = nx.complete_graph(6)
rng = np.random.default_rng(3)
xs_all = torch.as_tensor(0.02 + 0.01 * rng.standard_normal((6, N * N)), device="cuda")
yz = {e: (torch.as_tensor(0.001 * rng.standard_normal(N * N), device="cuda"),
          torch.as_tensor(0.02 + 0.001 * rng.standard_normal(N * N), device="cuda"))
      for e in [(min(a, b), max(a, b)) for a, b in G.edges()]}
res2 = {}
for V in (1, 2, 3, 4):
    P = make_subset_plan(G, 6, range(V))
    nb = NodeBatch(ops[0].geom, "float32", P, sinos, Q, 2.0, 0.02, 0.2, 10, 5, "iso", ph, 0, derive_z=False)
    for r, g in enumerate(P.local_nodes + P.halo_nodes):
        nb.x_ext[r].copy_(xs_all[g])
    for s, ge in enumerate(P.stored_edges):
        nb.y[s].copy_(yz[P.edges[ge]][0])
        nb.z[s].copy_(yz[P.edges[ge]][1])  # (stored z: derive_z=False)
    nb.node_update()
    nb.consensus()
    torch.cuda.synchronize()
    ek = [k for k, ge in enumerate(P.stored_edges) if P.edges[ge] == (0, 1)][0]
    res2[V] = (nb.x_local[0].cpu().numpy().copy(), nb.node_stats[0].cpu().numpy().copy(),
               nb.y[ek].cpu().numpy().copy(), nb.edge_stats[ek].cpu().numpy().copy())
    r0 = res2[1]
    print(f"edges V={V}: x equal {np.array_equal(res2[V][0], r0[0])} max|d|={np.abs(res2[V][0] - r0[0]).max():.3e}; "
          f"stats equal per column {[bool(a == b) for a, b in zip(res2[V][1], r0[1])]}; "
          f"y(0,1) equal {np.array_equal(res2[V][2], r0[2])}; edge stats equal {np.array_equal(res2[V][3], r0[3])}")
for V in (2, 3, 4, 8):
    print(f"no-edge stats V={V} per column equal: {[bool(a == b) for a, b in zip(res[V][1], res[1][1])]}")
