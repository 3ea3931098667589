"""Explicit-matrix operators: ``A_dense_list`` entries given as matrices.

The reference materialises each node's ODL ray transform as a dense float32 matrix
(``_to_dense_matrix``, /root/reference/block_2_load_odl_data.py:68-96), pickles the list
(/root/reference/block_3_graph_and_precisions.py:283-287) and its drivers hand that list
to ``decentralized_admm`` (/root/reference/block_7_main.py:16-22, 49-73).  The hot loop
uses it only through ``A.shape[1]``, ``A @ x``, ``A.T @ r`` and column norms
(/root/reference/block_6_admm_loop_ver2.py:26,145,193; block_3:20-23).

``MatrixOperator`` gives a matrix exactly that surface on the GPU: the library keeps A and
A^T as device CSR (``admm_ctx_create_matrix``, include/admm_tomo.h, ABI 4) and every
batch entry point -- the fused x-update, consensus, statistics -- runs unchanged with
the projector replaced by CSR products (``k_csr_fwd`` / ``k_back<..., CSR>``).  So a
reference-produced matrix (small N: dense A is 51 GB at 512^2) drives the same loop as
the matrix-free ``RayTransform``.

Matrices are read from files only through loaders that execute nothing from them:
``.npy`` (``np.load(allow_pickle=False)``) and ``.npz`` (a scipy.sparse ``save_npz``
archive or plain arrays, also ``allow_pickle=False``).  Pickles are refused.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import os

import numpy as np

from . import _lib
from .geometry import _torch, current_stream_handle, default_device, get_ctx

__all__ = ["MatrixGeometry", "MatrixOperator", "as_operators", "load_matrix", "load_matrix_list",
           "matrix_to_csr"]


def matrix_to_csr(A):
    """(m, n, indptr int64, indices int32, values float64) of a dense numpy / torch matrix
    or any scipy.sparse matrix.  Explicit zeros are dropped; column indices sorted."""
    import scipy.sparse as sp
    torch = _torch()
    if isinstance(A, torch.Tensor):
        A = A.detach().cpu().numpy()
    if sp.issparse(A):
        M = sp.csr_matrix(A, dtype=np.float64)
    else:
        a = np.asarray(A)
        if a.ndim != 2:
            raise ValueError(f"a matrix must be 2-D, got shape {a.shape}")
        M = sp.csr_matrix(a.astype(np.float64, copy=False))
    M.sum_duplicates()
    M.eliminate_zeros()
    M.sort_indices()
    m, n = M.shape
    if M.nnz >= (1 << 31):
        raise ValueError("matrix has >= 2^31 nonzeros")
    return (m, n, np.ascontiguousarray(M.indptr, dtype=np.int64),
            np.ascontiguousarray(M.indices, dtype=np.int32), np.ascontiguousarray(M.data, dtype=np.float64))


class MatrixGeometry:
    """The 'geometry' of an explicit-matrix context: image side N, m sinogram rows and the
    host CSR of A.  Equal (and hashed) by content digest, so identical matrices share one
    device context."""

    def __init__(self, N: int, m: int, indptr, indices, values):
        self.N = int(N)
        self.m = int(m)
        self.n = self.N * self.N
        self.indptr, self.indices, self.values = indptr, indices, values
        h = hashlib.blake2b(digest_size=16)
        for a in (np.array([self.N, self.m], dtype=np.int64), indptr, indices, values):
            h.update(np.ascontiguousarray(a).tobytes())
        self.digest = h.hexdigest()

    # the C context's one-"angle" layout (admm_ctx_create_matrix: n_det = m): a sinogram of a
    # matrix operator is its m rows (make_sinograms returns it flat)
    n_angles = 1

    @property
    def n_det(self) -> int:
        return self.m

    def __eq__(self, other):
        return isinstance(other, MatrixGeometry) and other.digest == self.digest

    def __hash__(self):
        return hash(("matrix", self.digest))

    def __repr__(self):
        return f"MatrixGeometry(N={self.N}, m={self.m}, nnz={len(self.indices)}, {self.digest[:8]})"

    def create_ctx(self, lib, dtype: str, device: int, max_images: int):
        """admm_ctx_create_matrix (include/admm_tomo.h)."""
        h = C.c_void_p()
        code = _lib.ADMM_DTYPE_F64 if dtype == "float64" else _lib.ADMM_DTYPE_F32
        _lib.check(lib.admm_ctx_create_matrix(
            C.byref(h), self.N, self.m, len(self.indices), self.indptr.ctypes.data_as(C.c_void_p),
            self.indices.ctypes.data_as(C.c_void_p), self.values.ctypes.data_as(C.c_void_p), code,
            max_images, device), "admm_ctx_create_matrix")
        return h


class MatrixOperator:
    """One node's operator given as an explicit (m x N^2) matrix; the drop-in for an entry of
    the reference's ``A_dense_list``.  ``A @ x`` / ``A.T @ y`` take numpy arrays or torch
    tensors of shape (n,) / (k, n) like ``RayTransform``; rows of A are sinogram entries in
    the reference's angle-major order, columns C-order pixels."""

    def __init__(self, A=None, N: int | None = None, dtype: str = "float32", device: int | None = None,
                 geom: MatrixGeometry | None = None):
        if dtype not in ("float32", "float64"):
            raise ValueError("dtype must be float32 or float64")
        if geom is None:
            if A is None:
                raise ValueError("give a matrix or a MatrixGeometry")
            m, n, indptr, indices, values = matrix_to_csr(A)
            Nn = int(round(n ** 0.5)) if N is None else int(N)
            if Nn * Nn != n:
                raise ValueError(f"matrix has {n} columns, not N*N for N={Nn}")
            geom = MatrixGeometry(Nn, m, indptr, indices, values)
        elif N is not None and int(N) != geom.N:
            raise ValueError(f"N={N} does not match the matrix geometry's N={geom.N}")
        self.geom = geom
        self.dtype = dtype
        self.device = default_device() if device is None else int(device)
        self.shape = (geom.m, geom.n)
        self._adjoint = False

    @property
    def T(self) -> "MatrixOperator":
        a = MatrixOperator(geom=self.geom, dtype=self.dtype, device=self.device)
        a._adjoint = not self._adjoint
        a.shape = (self.shape[1], self.shape[0])
        return a

    def __matmul__(self, x):
        return self.apply(x)

    @property
    def ctx(self):
        return get_ctx(self.geom, self.dtype, self.device)

    # the operator entry points are the same C functions as RayTransform's
    def apply(self, x):
        from .geometry import RayTransform
        return RayTransform.apply(self, x)

    def _tdtype(self):
        torch = _torch()
        return torch.float64 if self.dtype == "float64" else torch.float32

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


def _is_operator(A) -> bool:
    from .geometry import RayTransform
    return isinstance(A, (RayTransform, MatrixOperator))


def as_operators(A_list, N: int | None = None, dtype: str = "float32", device: int | None = None):
    """``A_dense_list`` -> operators: RayTransform / MatrixOperator entries pass through,
    matrices (dense numpy / torch, scipy.sparse) become MatrixOperators; equal matrices share
    one MatrixGeometry (one device context).  float32 samples by default, as the reference
    stores A (block_2_load_odl_data.py:84,96)."""
    out, seen = [], {}
    for A in A_list:
        if _is_operator(A):
            out.append(A)
            continue
        key = id(A)
        if key not in seen:
            m, n, indptr, indices, values = matrix_to_csr(A)
            Nn = int(round(n ** 0.5)) if N is None else int(N)
            if Nn * Nn != n:
                raise ValueError(f"matrix has {n} columns, not N*N for N={Nn}")
            seen[key] = MatrixGeometry(Nn, m, indptr, indices, values)
        out.append(MatrixOperator(geom=seen[key], dtype=dtype, device=device))
    return out


def load_matrix(path: str):
    """One matrix from ``.npy`` (dense) or ``.npz`` (scipy.sparse save_npz, or a single dense
    array); nothing in the file is executed (allow_pickle=False)."""
    ext = os.path.splitext(path)[1].lower()
    if ext == ".npy":
        return np.load(path, allow_pickle=False)
    if ext == ".npz":
        with np.load(path, allow_pickle=False) as z:
            keys = set(z.files)
            if {"data", "indices", "indptr", "shape"} <= keys:
                import scipy.sparse as sp
                return sp.load_npz(path)
            if len(keys) == 1:
                return z[next(iter(keys))]
        raise ValueError(f"{path}: expected a scipy.sparse archive or one array")
    raise ValueError(f"{path}: only .npy / .npz are loaded (pickles are not unpickled)")


def load_matrix_list(path: str):
    """``A_dense_list`` from ``.npy`` ([V, m, n] dense stack) or ``.npz`` (arrays named
    ``A_0``, ``A_1``, ... or ``arr_0``, ...; dense only), allow_pickle=False."""
    ext = os.path.splitext(path)[1].lower()
    if ext == ".npy":
        a = np.load(path, allow_pickle=False)
        if a.ndim != 3:
            raise ValueError(f"{path}: expected a [V, m, n] stack, got shape {a.shape}")
        return [a[i] for i in range(a.shape[0])]
    if ext == ".npz":
        with np.load(path, allow_pickle=False) as z:
            names = sorted(z.files, key=lambda s: (len(s), s))
            return [z[k] for k in names]
    raise ValueError(f"{path}: only .npy / .npz are loaded (pickles are not unpickled)")
