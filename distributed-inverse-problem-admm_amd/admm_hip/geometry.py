"""Parallel-beam geometry and the matrix-free ray transform (product path).

``RayTransform`` is the drop-in for one entry of the reference's
``A_dense_list`` (block_2_load_odl_data.py:68-96 materialises ODL's
RayTransform as a dense (m x n) float32 matrix).  The reference's hot loop uses
that matrix only through ``A.shape[1]``, ``A @ x`` and ``A.T @ r``
(block_6_admm_loop_ver2.py:26,145,193) and column norms
(block_3_graph_and_precisions.py:20-23); this object provides exactly those,
computed by the HIP projector (csrc/kernels.hpp k_fwd / k_back).  No dense
matrix is ever formed (51 GB at 512^2).
"""
from __future__ import annotations

import ctypes as C
import math
import threading
from dataclasses import dataclass

import numpy as np

from . import _lib


@dataclass(frozen=True)
class ParallelBeamGeometry:
    """ODL Parallel2dGeometry of block_2_load_odl_data.py:16-65.

    space ``uniform_discr([-1,-1], [1,1], [N,N])``; angles
    ``uniform_partition(angle_min, angle_max, n_angles)`` midpoints;
    detector ``uniform_partition(-w/2, w/2, N)`` with w = 2*det_width_factor.
    """

    N: int
    n_angles: int
    det_width_factor: float = 1.0
    angle_min: float = 0.0
    angle_max: float = math.pi

    @property
    def n_det(self) -> int:
        return self.N  # det_pixels = N (block_2_load_odl_data.py:44)

    @property
    def n(self) -> int:
        return self.N * self.N

    @property
    def m(self) -> int:
        return self.n_angles * self.n_det

    def to_c(self) -> _lib.Geom:
        w = 2.0 * self.det_width_factor
        return _lib.Geom(self.N, self.n_angles, self.n_det, 0, float(self.angle_min),
                         float(self.angle_max), -w / 2.0, w / 2.0)


def split_angles(angles_total: int, num_nodes: int) -> list[int]:
    """block_2_load_odl_data.py:35-38."""
    per = [angles_total // num_nodes] * num_nodes
    for i in range(angles_total % num_nodes):
        per[i] += 1
    return per


def _torch():
    import torch  # local import: torch is plumbing (device memory, streams)
    return torch


def default_device() -> int:
    """The calling process's current HIP device (torch.cuda.current_device()): with one
    process per GPU and ``torch.cuda.set_device(local_rank)`` first, every operator a rank
    builds lands on its own GPU.  0 when no GPU is visible (host-only logic, tests)."""
    torch = _torch()
    return int(torch.cuda.current_device()) if torch.cuda.is_available() else 0


def current_stream_handle(device=None) -> int:
    torch = _torch()
    return int(torch.cuda.current_stream(device).cuda_stream)


class _Ctx:
    """One C context (geometry tables + scratch) per (geometry, dtype, device); the
    geometry may also be an explicit matrix (matrix.MatrixGeometry)."""

    def __init__(self, geom, dtype: str, device: int, max_images: int = 64):
        self.lib = _lib.load()
        # the library keeps 32-bit element offsets per batch: cap the image count so
        # max_images x max(n, m) x 8 bytes stays below 2^31 (apply() splits larger batches)
        max_images = max(1, min(max_images, ((1 << 31) - 1) // (8 * max(geom.n, geom.m))))
        self.geom = geom
        self.dtype = dtype
        self.device = device
        if hasattr(geom, "create_ctx"):  # explicit matrix (matrix.MatrixGeometry)
            h = geom.create_ctx(self.lib, dtype, device, max_images)
        else:
            h = C.c_void_p()
            g = geom.to_c()
            code = _lib.ADMM_DTYPE_F64 if dtype == "float64" else _lib.ADMM_DTYPE_F32
            _lib.check(self.lib.admm_ctx_create(C.byref(h), C.byref(g), code, max_images, device),
                       "admm_ctx_create")
        self.h = h
        self.max_images = max_images

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            try:
                self.lib.admm_ctx_destroy(h)
            except Exception:  # pragma: no cover
                pass
            self.h = None


_ctx_lock = threading.Lock()
_ctx_cache: dict = {}


def get_ctx(geom: ParallelBeamGeometry, dtype: str, device: int) -> _Ctx:
    key = (geom, dtype, device)
    with _ctx_lock:
        c = _ctx_cache.get(key)
        if c is None:
            c = _Ctx(geom, dtype, device)
            _ctx_cache[key] = c
        return c


class RayTransform:
    """Matrix-free Joseph ray transform of one node (the ``A_i`` of the reference).

    ``A @ x`` accepts a numpy array or a torch tensor of shape (n,) or (k, n)
    (k images) and returns the same kind; ``A.T @ y`` is the exact adjoint.
    """

    def __init__(self, geom: ParallelBeamGeometry, dtype: str = "float32", device: int | None = None):
        if dtype not in ("float32", "float64"):
            raise ValueError("dtype must be float32 or float64")
        self.geom = geom
        self.dtype = dtype
        self.device = default_device() if device is None else int(device)
        self.shape = (geom.m, geom.n)
        self._adjoint = False

    # -- reference surface -------------------------------------------------
    @property
    def T(self) -> "RayTransform":
        a = RayTransform(self.geom, self.dtype, self.device)
        a._adjoint = not self._adjoint
        a.shape = (self.shape[1], self.shape[0])
        return a

    def __matmul__(self, x):
        return self.apply(x)

    # ----------------------------------------------------------------------
    @property
    def ctx(self) -> _Ctx:
        return get_ctx(self.geom, self.dtype, self.device)

    def _tdtype(self):
        torch = _torch()
        return torch.float64 if self.dtype == "float64" else torch.float32

    def apply(self, x):
        torch = _torch()
        is_np = not isinstance(x, torch.Tensor)
        dev = torch.device("cuda", self.device)
        xt = torch.as_tensor(np.asarray(x) if is_np else x)
        squeeze = xt.dim() == 1
        if squeeze:
            xt = xt.unsqueeze(0)
        if xt.shape[-1] != self.shape[1]:
            raise ValueError(f"operand has {xt.shape[-1]} entries, operator expects {self.shape[1]}")
        xt = xt.to(device=dev, dtype=self._tdtype()).contiguous()
        k = xt.shape[0]
        out = torch.empty((k, self.shape[0]), device=dev, dtype=self._tdtype())
        ctx = self.ctx
        s = current_stream_handle(dev)
        fn = ctx.lib.admm_project_adj if self._adjoint else ctx.lib.admm_project_fwd
        name = "admm_project_adj" if self._adjoint else "admm_project_fwd"
        for c0 in range(0, k, ctx.max_images):
            c1 = min(k, c0 + ctx.max_images)
            _lib.check(fn(ctx.h, C.c_void_p(xt[c0:c1].data_ptr()), C.c_void_p(out[c0:c1].data_ptr()),
                          c1 - c0, C.c_void_p(s)), name)
        if squeeze:
            out = out[0]
        if is_np:
            return out.double().cpu().numpy() if np.asarray(x).dtype == np.float64 else out.cpu().numpy()
        return out

    def column_norms_sq(self, as_numpy: bool = True):
        """W[p] = max(sum_r A[r,p]^2, 1e-12)  (make_precisions, block_3:20-23)."""
        torch = _torch()
        dev = torch.device("cuda", self.device)
        W = torch.empty(self.geom.n, device=dev, dtype=torch.float64)
        ctx = self.ctx
        _lib.check(ctx.lib.admm_column_norms_sq(ctx.h, C.c_void_p(W.data_ptr()),
                                                C.c_void_p(current_stream_handle(dev))),
                   "admm_column_norms_sq")
        return W.cpu().numpy() if as_numpy else W

    def __repr__(self) -> str:
        t = ".T" if self._adjoint else ""
        return f"RayTransform{t}(N={self.geom.N}, angles={self.geom.n_angles}, {self.dtype})"
