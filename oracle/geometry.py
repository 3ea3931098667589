"""Oracle: parallel-beam geometry, Joseph ray transform, phantom, analytic Radon.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Geometry restated from /root/reference/block_2_load_odl_data.py:16-65:
  * image space ``uniform_discr([-1,-1], [1,1], [N,N])`` (:23-28): pixel size
    h = 2/N, pixel centres x_i = -1 + (i+1/2) h, axis 0 = x, axis 1 = y;
  * angles ``uniform_partition(0, pi, a)`` (:51) -> midpoints (t+1/2) pi / a;
    every node spans the full half circle with its own ``a`` angles;
  * detector ``uniform_partition(-w/2, w/2, N)`` (:42-44, :52), w = 2*det_width_factor.
ODL Parallel2dGeometry defaults: detector axis at angle theta is
(cos theta, sin theta) and rays run along (-sin theta, cos theta), so detector
coordinate s sees the line  x cos(theta) + y sin(theta) = s.

Discretisation (the build's choice; ODL's backend is not available here):
Joseph's method.  In pixel-index units (p = x/h + c0, c0 = (N-1)/2) a ray
(theta, s) satisfies (p_x - c0) cos + (p_y - c0) sin = s/h.  If |cos| >= |sin|
("case A") we step over axis-1 index j and linearly interpolate along axis 0;
otherwise ("case B") we step over axis-0 index i and interpolate along axis 1.
Each step contributes the interpolated value times the path length h/|alpha|
(alpha = cos in case A, sin in case B).  Pixels outside the grid are zero.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import scipy.sparse as sp


@dataclass(frozen=True)
class Geometry:
    """2-D parallel-beam geometry of one graph node (block_2_load_odl_data.py:16-65)."""

    N: int
    n_angles: int
    det_width_factor: float = 1.0  # block_2_load_odl_data.py:16,42

    @property
    def n_det(self) -> int:
        return self.N  # det_pixels = N  (block_2_load_odl_data.py:44)

    @property
    def h(self) -> float:
        return 2.0 / self.N

    @property
    def h_det(self) -> float:
        return 2.0 * self.det_width_factor / self.n_det

    @property
    def angles(self) -> np.ndarray:
        # uniform_partition(0, pi, a) midpoints (block_2_load_odl_data.py:51)
        t = np.arange(self.n_angles, dtype=np.float64)
        return (t + 0.5) * math.pi / self.n_angles

    @property
    def det_centers(self) -> np.ndarray:
        # uniform_partition(-w/2, w/2, N) midpoints (block_2_load_odl_data.py:52)
        w = 2.0 * self.det_width_factor
        k = np.arange(self.n_det, dtype=np.float64)
        return -w / 2.0 + (k + 0.5) * self.h_det

    @property
    def shape(self) -> tuple[int, int]:
        return (self.n_angles * self.n_det, self.N * self.N)


def split_angles(angles_total: int, num_nodes: int) -> list[int]:
    """Per-node angle counts, block_2_load_odl_data.py:31-38."""
    per = [angles_total // num_nodes] * num_nodes
    for i in range(angles_total % num_nodes):
        per[i] += 1
    return per


def default_angles_total(N: int) -> int:
    """block_2_load_odl_data.py:31-33: max(180, 3N)."""
    return max(180, 3 * N)


def joseph_matrix(geom: Geometry, dtype=np.float64, angles=None) -> sp.csr_matrix:
    """Joseph ray transform of ``geom`` as a CSR matrix (m x n).

    Row r = t*n_det + k (angle-major, C order, as the flattened sinogram of
    block_6_admm_loop_ver2.py:46); column = C-order pixel i*N + j.
    ``angles`` (indices into the geometry's angle list) keeps only those angles'
    rows, in the given order (len(angles)*n_det rows) -- large-N spot checks.
    """
    N = geom.N
    c0 = 0.5 * (N - 1)
    th = geom.angles
    cs, sn = np.cos(th), np.sin(th)
    s_idx = geom.det_centers / geom.h  # detector coordinate in pixel units
    rows_all, cols_all, vals_all = [], [], []
    tsel = np.arange(geom.n_angles) if angles is None else np.asarray(angles, dtype=np.int64)
    T, K = np.meshgrid(tsel, np.arange(geom.n_det), indexing="ij")
    R, _ = np.meshgrid(np.arange(len(tsel)), np.arange(geom.n_det), indexing="ij")
    T = T.ravel()
    K = K.ravel()
    R = R.ravel()
    caseA = np.abs(cs[T]) >= np.abs(sn[T])
    alpha = np.where(caseA, cs[T], sn[T])
    beta = np.where(caseA, sn[T], cs[T])
    L = geom.h / np.abs(alpha)
    sk = s_idx[K]
    row = R * geom.n_det + K
    for m in range(N):
        l = c0 + (sk - (m - c0) * beta) / alpha
        i0 = np.floor(l)
        w = l - i0
        i0 = i0.astype(np.int64)
        for off, wt in ((0, 1.0 - w), (1, w)):
            li = i0 + off
            ok = (li >= 0) & (li < N) & (wt > 0)
            if not np.any(ok):
                continue
            lv = li[ok]
            pix = np.where(caseA[ok], lv * N + m, m * N + lv)
            rows_all.append(row[ok])
            cols_all.append(pix)
            vals_all.append((wt * L)[ok])
    rows = np.concatenate(rows_all)
    cols = np.concatenate(cols_all)
    vals = np.concatenate(vals_all).astype(dtype)
    A = sp.coo_matrix((vals, (rows, cols)), shape=(len(tsel) * geom.n_det, N * N)).tocsr()
    A.sum_duplicates()
    return A


def joseph_adjoint_gather(geom: Geometry, y: np.ndarray) -> np.ndarray:
    """Pixel-driven adjoint restated independently of :func:`joseph_matrix`.

    For pixel (i, j) and angle t the fractional bin is
    k_f = (c0 + (i-c0) cos + (j-c0) sin) mapped to detector index; the two bins
    floor(k_f), floor(k_f)+1 receive weight max(0, 1 - |k-k_f| * (h_det/h)/|alpha|)
    times h/|alpha|.  This is exactly the transpose of the Joseph weights in
    exact arithmetic; the HIP adjoint evaluates this formula.
    """
    N = geom.N
    c0 = 0.5 * (N - 1)
    y = np.asarray(y, dtype=np.float64).reshape(geom.n_angles, geom.n_det)
    I, J = np.meshgrid(np.arange(N), np.arange(N), indexing="ij")
    I = I.ravel().astype(np.float64) - c0
    J = J.ravel().astype(np.float64) - c0
    out = np.zeros(N * N)
    w_det = 2.0 * geom.det_width_factor
    ratio = geom.h_det / geom.h
    for t, th in enumerate(geom.angles):
        c, s = math.cos(th), math.sin(th)
        alpha = c if abs(c) >= abs(s) else s
        L = geom.h / abs(alpha)
        s_pix = I * c + J * s  # detector coordinate in pixel units
        kf = (s_pix * geom.h + w_det / 2.0) / geom.h_det - 0.5
        k0 = np.floor(kf)
        f = kf - k0
        k0 = k0.astype(np.int64)
        for off, dist in ((0, f), (1, 1.0 - f)):
            k = k0 + off
            wt = np.maximum(0.0, 1.0 - dist * ratio / abs(alpha)) * L
            ok = (k >= 0) & (k < geom.n_det) & (wt > 0)
            out[ok] += wt[ok] * y[t, k[ok]]
    return out


# ---------------------------------------------------------------------------
# Phantom and analytic Radon transform (geometry pin)
# ---------------------------------------------------------------------------

# Modified Shepp-Logan (Toft), [value, semi-axis a, semi-axis b, x0, y0, phi_deg]
SHEPP_LOGAN_MODIFIED = np.array(
    [
        [1.00, 0.6900, 0.9200, 0.0000, 0.0000, 0.0],
        [-0.80, 0.6624, 0.8740, 0.0000, -0.0184, 0.0],
        [-0.20, 0.1100, 0.3100, 0.2200, 0.0000, -18.0],
        [-0.20, 0.1600, 0.4100, -0.2200, 0.0000, 18.0],
        [0.10, 0.2100, 0.2500, 0.0000, 0.3500, 0.0],
        [0.10, 0.0460, 0.0460, 0.0000, 0.1000, 0.0],
        [0.10, 0.0460, 0.0460, 0.0000, -0.1000, 0.0],
        [0.10, 0.0460, 0.0230, -0.0800, -0.6050, 0.0],
        [0.10, 0.0230, 0.0230, 0.0000, -0.6060, 0.0],
        [0.10, 0.0230, 0.0460, 0.0600, -0.6050, 0.0],
    ]
)


def shepp_logan(N: int, supersample: int = 1) -> np.ndarray:
    """Modified Shepp-Logan on [-1,1]^2, array[i, j] <-> (x_i, y_j)."""
    return ellipse_phantom(N, SHEPP_LOGAN_MODIFIED, supersample)


def ellipse_phantom(N: int, table, supersample: int = 1) -> np.ndarray:
    """Sum of ellipses [value, a, b, x0, y0, phi_deg] on [-1,1]^2, pixel-averaged."""
    h = 2.0 / N
    ss = supersample
    sub = (np.arange(ss) + 0.5) / ss - 0.5
    xc = -1.0 + (np.arange(N) + 0.5) * h
    X = (xc[:, None] + sub[None, :] * h).ravel()
    XX, YY = np.meshgrid(X, X, indexing="ij")
    img = np.zeros_like(XX)
    for v, a, b, x0, y0, phi in table:
        p = math.radians(phi)
        xr = (XX - x0) * math.cos(p) + (YY - y0) * math.sin(p)
        yr = -(XX - x0) * math.sin(p) + (YY - y0) * math.cos(p)
        img += v * ((xr / a) ** 2 + (yr / b) ** 2 <= 1.0)
    img = img.reshape(N, ss, N, ss).mean(axis=(1, 3))
    return img


def shepp_logan_radon(geom: Geometry) -> np.ndarray:
    """Analytic line integrals of :func:`shepp_logan` for ``geom`` (a, n_det)."""
    return ellipse_radon(geom, SHEPP_LOGAN_MODIFIED)


def ellipse_radon(geom: Geometry, table) -> np.ndarray:
    """Analytic line integrals over the lines x cos(t) + y sin(t) = s (a, n_det)."""
    th = geom.angles[:, None]
    s = geom.det_centers[None, :]
    out = np.zeros((geom.n_angles, geom.n_det))
    for v, a, b, x0, y0, phi in table:
        p = math.radians(phi)
        sp_ = s - (x0 * np.cos(th) + y0 * np.sin(th))
        d2 = (a * np.cos(th - p)) ** 2 + (b * np.sin(th - p)) ** 2
        rad = d2 - sp_**2
        out += np.where(rad > 0, 2.0 * v * a * b * np.sqrt(np.maximum(rad, 0.0)) / d2, 0.0)
    return out
