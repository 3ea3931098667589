"""Oracle: TV operators.  TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates /root/reference/block_4_tv_helpers.py:
  * ``grad``  = ``_grad_forward_2d_from_vec`` (:17-23): C-order X, forward
    differences, gx[N-1,:] = 0, gy[:,N-1] = 0.
  * ``div_t`` = the exact adjoint K^T of ``grad``.  The reference's
    ``_div_backward_2d_to_vec`` (:25-35) has the wrong sign on its first/last
    row and column terms; this restatement uses the true adjoint
    (documented deviation).
  * ``subgrad`` = ``kt_subgrad_isotropic_tv_from_x`` (:37-46) with eps=1e-12,
    but with the exact adjoint.
  * ``tv_value`` = textbook isotropic TV sum_p ||(gx,gy)_p||_2 (the intent of
    the CVXPY atom ``isotropic_tv_on_vector`` :5-14, without its F-order
    pairing defect); anisotropic = sum |gx|+|gy|.
"""
from __future__ import annotations

import numpy as np


def grad(x: np.ndarray, N: int) -> tuple[np.ndarray, np.ndarray]:
    X = x.reshape(N, N)
    gx = np.zeros_like(X)
    gy = np.zeros_like(X)
    gx[:-1, :] = X[1:, :] - X[:-1, :]
    gy[:, :-1] = X[:, 1:] - X[:, :-1]
    return gx.reshape(-1), gy.reshape(-1)


def div_t(px: np.ndarray, py: np.ndarray, N: int) -> np.ndarray:
    """Exact K^T:  (K^T p)[i,j] = px[i-1,j]*[i>=1] - px[i,j]*[i<=N-2] + (same in j)."""
    PX = px.reshape(N, N)
    PY = py.reshape(N, N)
    out = np.zeros((N, N), dtype=np.result_type(px, py))
    out[1:, :] += PX[:-1, :]
    out[:-1, :] -= PX[:-1, :]
    out[:, 1:] += PY[:, :-1]
    out[:, :-1] -= PY[:, :-1]
    return out.reshape(-1)


def ktk(x: np.ndarray, N: int) -> np.ndarray:
    gx, gy = grad(x, N)
    return div_t(gx, gy, N)


def shrink(ux: np.ndarray, uy: np.ndarray, tau: float, kind: str = "iso"):
    if kind == "iso":
        s = np.sqrt(ux * ux + uy * uy)
        f = np.where(s > tau, (s - tau) / np.where(s > 0, s, 1.0), 0.0)
        return f * ux, f * uy
    if kind == "aniso":
        return (np.sign(ux) * np.maximum(np.abs(ux) - tau, 0.0),
                np.sign(uy) * np.maximum(np.abs(uy) - tau, 0.0))
    raise ValueError(kind)


def tv_value(x: np.ndarray, N: int, kind: str = "iso") -> float:
    gx, gy = grad(x, N)
    if kind == "iso":
        return float(np.sum(np.sqrt(gx * gx + gy * gy)))
    return float(np.sum(np.abs(gx) + np.abs(gy)))


def subgrad(x: np.ndarray, N: int, kind: str = "iso", eps: float = 1e-12) -> np.ndarray:
    """K^T p with p a TV subgradient at Kx (block_4_tv_helpers.py:37-46)."""
    gx, gy = grad(x, N)
    if kind == "iso":
        mag = np.sqrt(gx * gx + gy * gy)
        m = mag > eps
        safe = np.where(m, mag, 1.0)
        px = np.where(m, gx / safe, 0.0)
        py = np.where(m, gy / safe, 0.0)
    else:
        px = np.where(np.abs(gx) > eps, np.sign(gx), 0.0)
        py = np.where(np.abs(gy) > eps, np.sign(gy), 0.0)
    return div_t(px, py, N)
