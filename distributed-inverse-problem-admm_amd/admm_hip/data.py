"""Problem setup on the GPU: phantom, per-node sinograms, precisions.

* ``shepp_logan``   -- modified Shepp-Logan on [-1,1]^2 (the benchmark phantom of
  SURVEY.md 8d; the reference itself uses randIm/ConstIm, Gen_Sino_Partitioned.py:5-122).
* ``make_sinograms`` -- b_i = A_i x + sigma * N(0,1)
  (block_2_load_odl_data.py:148-153), noise from a seeded on-device generator
  (seed base 1000 + i; the reference is unseeded).
* ``make_precisions`` -- W_i[p] = max(||A_i[:,p]||^2, 1e-12) and the arithmetic /
  harmonic Q_ij provider of block_3_graph_and_precisions.py:11-43, with W from
  the matrix-free HIP kernel (admm_column_norms_sq) instead of dense column sums.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .geometry import RayTransform

# [value, semi-axis a, semi-axis b, x0, y0, phi_deg]  (modified Shepp-Logan, Toft)
SHEPP_LOGAN_MODIFIED = (
    (1.00, 0.6900, 0.9200, 0.0000, 0.0000, 0.0),
    (-0.80, 0.6624, 0.8740, 0.0000, -0.0184, 0.0),
    (-0.20, 0.1100, 0.3100, 0.2200, 0.0000, -18.0),
    (-0.20, 0.1600, 0.4100, -0.2200, 0.0000, 18.0),
    (0.10, 0.2100, 0.2500, 0.0000, 0.3500, 0.0),
    (0.10, 0.0460, 0.0460, 0.0000, 0.1000, 0.0),
    (0.10, 0.0460, 0.0460, 0.0000, -0.1000, 0.0),
    (0.10, 0.0460, 0.0230, -0.0800, -0.6050, 0.0),
    (0.10, 0.0230, 0.0230, 0.0000, -0.6060, 0.0),
    (0.10, 0.0230, 0.0460, 0.0600, -0.6050, 0.0),
)


def shepp_logan(N: int, supersample: int = 4, device=None, dtype=torch.float64) -> torch.Tensor:
    """(N, N) phantom, array[i, j] <-> (x_i, y_j), pixel-averaged over ss^2 sub-samples."""
    dev = torch.device("cpu") if device is None else torch.device(device)
    h = 2.0 / N
    ss = supersample
    sub = (torch.arange(ss, dtype=torch.float64, device=dev) + 0.5) / ss - 0.5
    xc = -1.0 + (torch.arange(N, dtype=torch.float64, device=dev) + 0.5) * h
    X = (xc[:, None] + sub[None, :] * h).reshape(-1)
    XX, YY = torch.meshgrid(X, X, indexing="ij")
    img = torch.zeros_like(XX)
    for v, a, b, x0, y0, phi in SHEPP_LOGAN_MODIFIED:
        p = math.radians(phi)
        xr = (XX - x0) * math.cos(p) + (YY - y0) * math.sin(p)
        yr = -(XX - x0) * math.sin(p) + (YY - y0) * math.cos(p)
        img += v * (((xr / a) ** 2 + (yr / b) ** 2) <= 1.0).to(torch.float64)
    img = img.reshape(N, ss, N, ss).mean(dim=(1, 3))
    return img.to(dtype)


def make_sinograms(ops: list[RayTransform], phantom, noise_level: float = 0.005, seed: int = 1000):
    """Per-node noisy sinograms (a_i, N) on the operators' device, in the operators' dtype."""
    out = []
    for i, A in enumerate(ops):
        dev = torch.device("cuda", A.device)
        ph = torch.as_tensor(phantom).reshape(-1).to(device=dev)
        clean = A @ ph.to(torch.float64 if A.dtype == "float64" else torch.float32)
        gen = torch.Generator(device=dev)
        gen.manual_seed(seed + i)
        noise = torch.randn(clean.shape, generator=gen, device=dev, dtype=torch.float64)
        b = (clean.to(torch.float64) + noise_level * noise).to(clean.dtype)
        # (angles, detector bins) like the reference's sinograms; a matrix operator's rows flat
        out.append(b.reshape(-1) if hasattr(A.geom, "digest") else b.reshape(A.geom.n_angles, A.geom.n_det))
    return out


def ridge_ls(A, b, lam_ridge: float = 1e-3, max_iters: int = 2000, rtol: float = 1e-10):
    """argmin_x ||A x - b||^2 + lam_ridge ||x||^2 = (A^T A + lam I)^{-1} A^T b, by CG on the GPU.

    The legacy loader's aggregate reconstruction (/root/reference/block_2_test.py:83-88:
    ``np.linalg.solve(A_agg.T @ A_agg + 1e-3 I, A_agg.T @ b)`` on the dense n x n normal
    matrix).  The normal operator is applied matrix-free with float64 samples (a float32
    projector's rounding, amplified by the ridge system's conditioning, would show at the
    1e-4 level); stops when ||r|| <= rtol ||A^T b|| or after ``max_iters`` steps.
    Returns (x float64 (n,) tensor, iterations, relative residual)."""
    from .geometry import RayTransform
    Af = RayTransform(A.geom, "float64", A.device) if isinstance(A, RayTransform) else A
    dev = torch.device("cuda", Af.device)
    bt = torch.as_tensor(b).reshape(-1).to(device=dev, dtype=torch.float64)
    atb = Af.T @ bt
    x = torch.zeros_like(atb)
    r = atb.clone()
    p = r.clone()
    rs = float(r @ r)
    stop = (rtol ** 2) * rs
    it = 0
    while it < max_iters and rs > stop:
        Ap = Af.T @ (Af @ p) + lam_ridge * p
        alpha = rs / float(p @ Ap)
        x += alpha * p
        r -= alpha * Ap
        rs_new = float(r @ r)
        p = r + (rs_new / rs) * p
        rs = rs_new
        it += 1
    base = float(atb @ atb)
    return x, it, (rs / base) ** 0.5 if base > 0 else 0.0


class QProvider:
    """Q_ij provider of block_3_graph_and_precisions.py:26-39 (callable (i, j) -> (n,)).

    ``qslot_key(i, j)`` tells the device batch which pairs share one vector so
    identical Q_ij are stored once in HBM (all W_i are equal when every node
    has the same geometry).
    """

    def __init__(self, Wi_list, q_mode: str = "arithmetic", W_keys=None):
        if q_mode not in ("arithmetic", "harmonic"):
            raise ValueError("q_mode must be 'harmonic' or 'arithmetic'")
        self.Wi_list = Wi_list
        self.q_mode = q_mode
        self.W_keys = W_keys

    def __call__(self, i, j):
        eps = 1e-12
        wi, wj = self.Wi_list[i], self.Wi_list[j]
        if self.q_mode == "harmonic":
            q = (wi * wj) / (wi + wj)
        else:
            q = 0.5 * (wi + wj)
        return np.maximum(q, eps)

    def qslot_key(self, i, j):
        if self.W_keys is None:
            return None
        a, b = self.W_keys[i], self.W_keys[j]
        return (self.q_mode, min(a, b), max(a, b))


def make_precisions(ops: list[RayTransform], q_mode: str = "arithmetic"):
    """(Wi_list, Qij_diag) with W from the HIP kernel (block_3_graph_and_precisions.py:11-43).
    ``ops`` may also hold matrices (the reference's dense A_dense_list): matrix.as_operators."""
    from .matrix import as_operators
    cache, Wi_list, keys = {}, [], []
    for A in as_operators(ops):
        key = (A.geom, A.dtype, A.device)
        if key not in cache:
            cache[key] = (len(cache), A.column_norms_sq(as_numpy=True))
        k, W = cache[key]
        Wi_list.append(W)
        keys.append(k)
    return Wi_list, QProvider(Wi_list, q_mode, keys)
