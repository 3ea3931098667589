"""A/B probe: check_bitwise.py's problem (5-node ring, CHECK_N^2, 240 angles, 3 iterations)
on the library ADMM_TOMO_LIB names, against the CPU oracle: prints the relative errors."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "distributed-inverse-problem-admm_amd"), ROOT, os.path.join(ROOT, "tests")]
import networkx as nx  # noqa: E402
import numpy as np  # noqa: E402

from test_gpu_admm import rel, setup_problem  # noqa: E402
from block_6_admm_loop_ver2 import decentralized_admm  # noqa: E402
from oracle import admm as oadmm  # noqa: E402

N, V = int(os.environ.get("CHECK_N", "64")), 5
ops, ph, sinos, Wi, Q, A, sin_h = setup_problem(N, V, 240)
G = nx.cycle_graph(V)
x, h = decentralized_admm(ops, sinos, G, Wi, Q, N, lam_tv=0.02, rho=2.0, max_iters=3, eps_pri=0.0,
                          eps_dual=0.0, verbose=False, phantom_true=ph, write_params=False)
xo, ho = oadmm.decentralized_admm([A] * V, sin_h, G, Q, N, lam_tv=0.02, rho=2.0, max_iters=3, eps_pri=0.0,
                                  eps_dual=0.0, phantom_true=ph)
print(os.environ.get("ADMM_TOMO_LIB", "in-tree"), {k: f"{v:.2e}" for k, v in {
    "x": rel(np.stack(x), np.stack(xo)), "primal": rel(h["primal"], ho["primal"]),
    "mse": rel(h["mse_sino_total"], ho["mse_sino_total"]),
    "g": rel(np.stack(h["g_norm_history"]), np.stack(ho["g_norm_history"]))}.items()})
