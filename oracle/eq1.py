"""Oracle: the node objective eq.(1) solved independently of split Bregman, and an
a-posteriori optimality certificate.  TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

eq.(1) (block_5_node_problem.py:21-29, ADMM_Algo.pdf p.4):

    f(x) = 1/2 ||A x - b||^2 + lam TV(K x) + sum_j rho/2 sum_p q_ij[p] (x[p] - v_ij[p])^2
         = 1/2 x^T H x - g^T x + lam ||K x||_{2,1} + const,
    H = A^T A + rho diag(D),  g = A^T b + rho c,  D = sum_j q_ij,  c = sum_j q_ij v_ij

(block_6_admm_loop_ver2.py:137-146 builds exactly D and c for its stationarity check).
TV is the textbook one: isotropic sum_p ||(Kx)_p||_2 or
anisotropic sum_p |(Kx)_p,x| + |(Kx)_p,y|.

* ``pdhg_solve`` -- Chambolle-Pock primal-dual method, accelerated for the strongly
  convex quadratic (their Algorithm 2, gamma = lambda_min(H)), with the exact prox of the
  quadratic from one dense eigendecomposition of H (small N only).  Shares nothing with
  the split-Bregman/CG iteration of node_solver.py except the K stencil.
* ``certificate`` -- for any x and any dual field p with |p_pix| <= 1 (2-norm for iso,
  max-norm for aniso) the vector  r = H x - g + lam K^T p  and
  eps = lam (TV(Kx) - <p, Kx>) >= 0  give  lam p in d_eps(lam TV)(Kx), hence for every z
  f(z) >= f(x) + <r, z - x> - eps + m/2 ||z - x||^2  (m = lambda_min(H)), so
      ||x - x*|| <= (||r|| + sqrt(||r||^2 + 2 m eps)) / m,   f(x) - f(x*) <= ||r||^2/(2m) + eps.
  For a split-Bregman state the natural dual is p = mu e / lam (the shrink leaves
  |e| <= lam/mu, aligned with d where d != 0).
"""
from __future__ import annotations

import numpy as np

from . import tv as tvmod


def _project(px, py, kind):
    if kind == "iso":
        s = np.maximum(1.0, np.sqrt(px * px + py * py))
        return px / s, py / s
    return np.clip(px, -1.0, 1.0), np.clip(py, -1.0, 1.0)


def hessian(A, D, rho):
    """Dense H = A^T A + rho diag(D) (small N)."""
    Ad = A.toarray() if hasattr(A, "toarray") else np.asarray(A)
    return Ad.T @ Ad + rho * np.diag(np.asarray(D, dtype=np.float64))


def certificate(A, b, D, c, x, px, py, N, rho, lam, kind="iso", m=None, H=None):
    """(dist_bound, gap_bound, ||r||, eps) for the candidate x with dual field (px, py)."""
    px, py = _project(np.asarray(px, np.float64), np.asarray(py, np.float64), kind)
    if H is not None:
        r = H @ x - (A.T @ b + rho * c)
    else:
        r = A.T @ (A @ x - b) + rho * (D * x - c)
    r = r + lam * tvmod.div_t(px, py, N)
    gx, gy = tvmod.grad(x, N)
    eps = max(0.0, lam * (tvmod.tv_value(x, N, kind) - float(px @ gx + py @ gy)))
    if m is None:
        m = rho * float(np.min(D))  # lambda_min(A^T A) >= 0
    rn = float(np.linalg.norm(r))
    return (rn + np.sqrt(rn * rn + 2.0 * m * eps)) / m, rn * rn / (2.0 * m) + eps, rn, eps


def pdhg_solve(A, b, D, c, N, rho, lam, kind="iso", iters=20000, H=None):
    """Accelerated Chambolle-Pock for eq.(1).  Returns (x, px, py, m) with p = y / lam."""
    if H is None:
        H = hessian(A, D, rho)
    ev, Q = np.linalg.eigh(H)
    m = float(ev[0])
    g = np.asarray(A.T @ b + rho * c, dtype=np.float64)
    n = N * N
    x = np.zeros(n)
    xb = x.copy()
    yx = np.zeros(n)
    yy = np.zeros(n)
    tau = sig = 1.0 / np.sqrt(8.0)  # ||K||^2 <= 8
    for _ in range(iters):
        gx, gy = tvmod.grad(xb, N)
        yx, yy = _project((yx + sig * gx) / lam, (yy + sig * gy) / lam, kind)
        yx *= lam
        yy *= lam
        v = x - tau * tvmod.div_t(yx, yy, N) + tau * g
        xn = Q @ ((Q.T @ v) / (1.0 + tau * ev))
        th = 1.0 / np.sqrt(1.0 + 2.0 * m * tau)
        tau *= th
        sig /= th
        xb = xn + th * (xn - x)
        x = xn
    return x, yx / lam, yy / lam, m
