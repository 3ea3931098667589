"""Oracle: per-node x-update.  TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Objective (block_5_node_problem.py:21-29, ADMM_Algo.pdf eq.(1)):

    f(x) = 1/2 ||A x - b||^2 + lam * TV(x) + sum_j rho/2 sum_p q_ij[p] (x[p]-v_ij[p])^2

with D = sum_j q_ij and c = sum_j q_ij * v_ij (block_6_admm_loop_ver2.py:137-146).

The reference hands this to CVXPY+SCS (block_6_admm_loop_ver2.py:123).  The
build replaces it with a deterministic fixed-count split-Bregman iteration
(d ~ Kx, Bregman variable e, penalty mu), each x-subproblem

    (A^T A + rho D + mu K^T K) x = A^T b + rho c + mu K^T (d - e)

solved by ``cg_iters`` conjugate-gradient steps warm-started from the current
x.  The CG keeps its residual recursively across TV rounds
(r += mu K^T (w_new - w_old), w = d - e) and takes every scalar from ONE fused
reduction per step (the back-projector epilogue on the device):
p.Hp, r.Hp, Hp.Hp, r.r, r.p.  The step is the exact line search
alpha = r.p / p.Hp (equal to r.r / p.Hp in exact CG, but stable when
orthogonality is lost), and beta = ||r - alpha Hp||^2 / r.r with the numerator
from the identity rr - 2 alpha r.Hp + alpha^2 Hp.Hp -- exactly as the HIP path
(csrc/kernels.hpp k_back<BACK_H>, k_cg_update) does.  Scalars are float64; vectors are float64 by
default or float32 (``dtype``) to emulate the device arithmetic.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import tv as tvmod


@dataclass
class NodeParams:
    rho: float
    lam: float
    mu: float
    tv_iters: int = 10
    cg_iters: int = 5
    tv_kind: str = "iso"


@dataclass
class NodeState:
    x: np.ndarray
    dx: np.ndarray
    dy: np.ndarray
    ex: np.ndarray
    ey: np.ndarray

    @classmethod
    def zeros(cls, n: int, dtype=np.float64) -> "NodeState":
        z = lambda: np.zeros(n, dtype=dtype)  # noqa: E731
        return cls(z(), z(), z(), z(), z())


@dataclass
class NodeDiag:
    obj: float = 0.0
    mse_sino: float = 0.0
    g_norm: float = 0.0
    sb_res: float = 0.0  # ||A^T s + rho (D x - c) + mu K^T e||: stationarity with p = mu e / lam
    tv: float = 0.0
    quad: float = 0.0
    cg_rr: list = field(default_factory=list)


def assemble(qv_terms, n: int):
    """D = sum_j q_ij, c = sum_j q_ij * v_ij in neighbour order (block_6_admm_loop_ver2.py:137-146)."""
    D = np.zeros(n)
    c = np.zeros(n)
    for q, v in qv_terms:
        D += q
        c += q * v
    return D, c


def _dot(a, b) -> float:
    return float(np.dot(a.astype(np.float64), b.astype(np.float64)))


def node_update(A, Atb, b, D, c, qv_terms, st: NodeState, N: int, p: NodeParams,
                dtype=np.float64, AT=None) -> NodeDiag:
    """In-place fixed-count split-Bregman x-update of one node.

    ``A`` is a (sparse) matrix, ``AT`` its transpose (defaults to A.T).
    ``qv_terms`` = list of (q_ij, v_ij) for the objective's quadratic term.
    """
    AT = A.T if AT is None else AT
    cast = lambda v: np.asarray(v, dtype=dtype)  # noqa: E731
    rho, lam, mu = p.rho, p.lam, p.mu
    D = cast(D)
    c = cast(c)
    Atb = cast(Atb)

    def H(v):
        return cast(AT @ cast(A @ v)) + cast(rho * D * v) + cast(mu * tvmod.ktk(v, N))

    x = st.x
    wx = cast(st.dx - st.ex)
    wy = cast(st.dy - st.ey)
    r = cast(Atb + rho * c + mu * tvmod.div_t(wx, wy, N) - H(x))
    pvec = r.copy()
    diag = NodeDiag()
    for t in range(p.tv_iters):
        for _ in range(p.cg_iters):
            Hp = H(pvec)
            pHp = _dot(pvec, Hp)
            rHp = _dot(r, Hp)
            HpHp = _dot(Hp, Hp)
            rr = _dot(r, r)
            rp = _dot(r, pvec)
            alpha = rp / pHp if pHp != 0.0 else 0.0
            rr_new = rr - 2.0 * alpha * rHp + alpha * alpha * HpHp
            rr_new = max(rr_new, 0.0)
            beta = rr_new / rr if rr != 0.0 else 0.0
            x += cast(alpha * pvec)
            r -= cast(alpha * Hp)
            pvec = cast(r + beta * pvec)
            diag.cg_rr.append(rr)
        # TV (d, e) update: u = Kx + e, d = shrink(u, lam/mu), e = u - d
        gx, gy = tvmod.grad(x, N)
        ux = cast(gx + st.ex)
        uy = cast(gy + st.ey)
        dx, dy = tvmod.shrink(ux, uy, lam / mu, p.tv_kind)
        st.dx[:] = dx
        st.dy[:] = dy
        st.ex[:] = ux - st.dx
        st.ey[:] = uy - st.dy
        if t + 1 < p.tv_iters:
            nwx = cast(st.dx - st.ex)
            nwy = cast(st.dy - st.ey)
            r += cast(mu * tvmod.div_t(nwx - wx, nwy - wy, N))
            wx, wy = nwx, nwy
            pvec = r.copy()
    # Epilogue diagnostics (block_6_admm_loop_ver2.py:125-149,189-197)
    s = cast(A @ x) - cast(b)
    diag.mse_sino = _dot(s, s)
    g = cast(AT @ s) + cast(rho * (D * x - c)) + cast(lam * tvmod.subgrad(x, N, p.tv_kind))
    diag.g_norm = float(np.sqrt(_dot(g, g)))
    rsb = cast(AT @ s) + cast(rho * (D * x - c)) + cast(mu * tvmod.div_t(st.ex, st.ey, N))
    diag.sb_res = float(np.sqrt(_dot(rsb, rsb)))
    diag.tv = tvmod.tv_value(x.astype(np.float64), N, p.tv_kind)
    quad = 0.0
    for q, v in qv_terms:
        dv = x.astype(np.float64) - np.asarray(v, dtype=np.float64)
        quad += 0.5 * rho * float(np.sum(np.asarray(q, dtype=np.float64) * dv * dv))
    diag.quad = quad
    diag.obj = 0.5 * diag.mse_sino + lam * diag.tv + quad
    return diag


def objective(A, b, x, N, rho, lam, qv_terms, kind="iso") -> float:
    """Node objective eq.(1) (block_5_node_problem.py:21-29), float64."""
    s = A @ x - b
    val = 0.5 * float(s @ s) + lam * tvmod.tv_value(x, N, kind)
    for q, v in qv_terms:
        dv = x - v
        val += 0.5 * rho * float(np.sum(q * dv * dv))
    return val
