"""Generate tests/golden/*.npz from the CPU oracle (run: python tests/golden/make_golden.py).

The reference ships no golden vectors for this path and could
not be executed here, so these fixtures pin the oracle itself (regression
vectors) plus one independent physical pin: the analytic Radon transform of
the modified Shepp-Logan ellipses in ODL's Parallel2dGeometry convention.
"""
from __future__ import annotations

import os
import sys

import networkx as nx
import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import admm as oadmm  # noqa: E402
from oracle import node_solver as ons  # noqa: E402
from oracle import tv as otv  # noqa: E402
from oracle.geometry import Geometry, joseph_matrix, shepp_logan, shepp_logan_radon  # noqa: E402


def problem(N=16, V=3, a=12, seed=1000):
    A = joseph_matrix(Geometry(N, a))
    ph = shepp_logan(N, 4).ravel()
    sinos = [A @ ph + 0.005 * np.random.default_rng(seed + i).standard_normal(A.shape[0]) for i in range(V)]
    W = np.maximum(np.asarray(A.multiply(A).sum(axis=0)).ravel(), 1e-12)
    return A, ph, sinos, W


def main():
    out = {}
    # 1. projector fingerprint: A @ x0 and A^T @ y0 for seeded inputs, 16^2 x 12 angles
    A, ph, sinos, W = problem()
    rng = np.random.default_rng(42)
    x0 = rng.standard_normal(A.shape[1])
    y0 = rng.standard_normal(A.shape[0])
    out["proj_x0"] = x0
    out["proj_y0"] = y0
    out["proj_Ax0"] = A @ x0
    out["proj_ATy0"] = A.T @ y0
    out["proj_W"] = W
    # 2. analytic pin at 64^2 / 48 angles (discretisation error ~6e-2 rel, O(h))
    g = Geometry(64, 48)
    out["radon64_joseph"] = joseph_matrix(g) @ shepp_logan(64, 4).ravel()
    out["radon64_analytic"] = shepp_logan_radon(g).ravel()
    # 3. TV operators on a seeded 16^2 image
    xt = rng.standard_normal(256)
    gx, gy = otv.grad(xt, 16)
    out["tv_x"] = xt
    out["tv_gx"], out["tv_gy"] = gx, gy
    out["tv_div"] = otv.div_t(gx, gy, 16)
    out["tv_sub_iso"] = otv.subgrad(xt, 16, "iso")
    out["tv_sub_aniso"] = otv.subgrad(xt, 16, "aniso")
    sx, sy = otv.shrink(gx, gy, 0.3, "iso")
    out["tv_shrink_iso"] = np.stack([sx, sy])
    # 4. one node x-update (2 neighbour terms)
    b = sinos[0]
    q1, q2 = W, 1.5 * W
    v1, v2 = ph + 0.01, ph - 0.02
    st = ons.NodeState.zeros(256)
    d = ons.node_update(A, A.T @ b, b, q1 + q2, q1 * v1 + q2 * v2, [(q1, v1), (q2, v2)], st, 16,
                        ons.NodeParams(rho=2.0, lam=0.02, mu=0.2, tv_iters=4, cg_iters=3))
    out["node_b"] = b
    out["node_x"] = st.x
    out["node_obj"] = np.array([d.obj, d.mse_sino, d.g_norm, d.tv, d.quad])
    # 5. ADMM trajectory, 3-node ring, 4 iterations
    x, h = oadmm.decentralized_admm([A] * 3, sinos, nx.cycle_graph(3), lambda i, j: W, 16, lam_tv=0.02,
                                    rho=2.0, max_iters=4, eps_pri=0.0, eps_dual=0.0, phantom_true=ph,
                                    tv_iters=4, cg_iters=3)
    out["admm_sinos"] = np.stack(sinos)
    out["admm_x"] = np.stack(x)
    for k in ("primal", "dual", "obj_total", "mse_sino_total", "img_mse_total"):
        out[f"admm_{k}"] = np.asarray(h[k])
    np.savez_compressed(os.path.join(HERE, "oracle_golden.npz"), **out)
    print("wrote", os.path.join(HERE, "oracle_golden.npz"), sum(v.nbytes for v in out.values()), "bytes")


if __name__ == "__main__":
    main()
