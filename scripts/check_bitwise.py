"""Run one small ADMM solve (64^2 or CHECK_N^2, 5-node ring, 3 iterations, float32 samples) with
the library ADMM_TOMO_LIB points to and save x / histories; with --compare A.npz B.npz report
whether two runs are bitwise equal (A/B of code paths that must not change results)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "distributed-inverse-problem-admm_amd"), ROOT]
import numpy as np  # noqa: E402

if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    same = all(np.array_equal(a[k], b[k]) for k in a.files)
    diff = max(float(np.max(np.abs(a[k] - b[k]))) for k in a.files)
    print(f"bitwise equal: {same}  (max |diff| {diff:.3e})")
    sys.exit(0 if same else 1)

import networkx as nx  # noqa: E402
import torch  # noqa: E402

from admm_hip.data import make_precisions, make_sinograms, shepp_logan  # noqa: E402
from admm_hip.solver import make_operators  # noqa: E402
from block_6_admm_loop_ver2 import decentralized_admm  # noqa: E402

N, V = int(os.environ.get("CHECK_N", "64")), 5  # (N % 16 != 0: segments end in short chunks)
ops = make_operators(N, V, angles_total=240, device=0)
ph = shepp_logan(N)
sinos = make_sinograms(ops, ph, 0.005)
Wi, Q = make_precisions(ops)
x, h = decentralized_admm(ops, sinos, nx.cycle_graph(V), Wi, Q, N, lam_tv=0.02, rho=2.0, max_iters=3,
                          eps_pri=0.0, eps_dual=0.0, verbose=False, phantom_true=ph.numpy(), write_params=False)
np.savez(sys.argv[1], x=np.stack(x), primal=np.array(h["primal"]), dual=np.array(h["dual"]),
         g=np.stack(h["g_norm_history"]), mse=np.array(h["mse_sino_total"]))
torch.cuda.synchronize()
print("saved", sys.argv[1])
