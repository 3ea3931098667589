"""CPU: the explicit-matrix operator path (admm_hip/matrix.py) without a
GPU -- CSR conversion of every accepted matrix kind, the non-executing file loaders, content
identity of matrix geometries, and admm_ctx_create_matrix's argument checks (which run
before any HIP call)."""
import ctypes as C

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from admm_hip import _lib
from admm_hip.geometry import ParallelBeamGeometry, RayTransform
from admm_hip.matrix import (MatrixGeometry, MatrixOperator, as_operators, load_matrix, load_matrix_list,
                             matrix_to_csr)
from oracle.geometry import Geometry, joseph_matrix


def _ref():
    return joseph_matrix(Geometry(8, 12)).tocsr()


@pytest.mark.parametrize("kind", ["dense", "float32", "torch", "coo", "csc"])
def test_matrix_to_csr_every_kind(kind):
    A = _ref()
    src = {"dense": A.toarray(), "float32": A.toarray().astype(np.float32), "torch": torch.as_tensor(A.toarray()),
           "coo": A.tocoo(), "csc": A.tocsc()}[kind]
    m, n, indptr, indices, values = matrix_to_csr(src)
    assert (m, n) == A.shape and indptr.dtype == np.int64 and indices.dtype == np.int32
    B = sp.csr_matrix((values, indices, indptr), shape=(m, n))
    tol = 1e-7 if kind == "float32" else 0.0
    assert abs(B - A).max() <= tol
    assert np.all(values != 0)  # explicit zeros dropped
    for r in range(m):  # sorted column indices per row
        assert np.all(np.diff(indices[indptr[r]:indptr[r + 1]]) > 0)


def test_geometry_identity_is_content():
    A = _ref()
    g1 = MatrixGeometry(8, A.shape[0], *matrix_to_csr(A)[2:])
    g2 = MatrixGeometry(8, A.shape[0], *matrix_to_csr(A.toarray().copy())[2:])
    A2 = A.copy()
    A2[0, A2[0].indices[0]] *= 2
    g3 = MatrixGeometry(8, A.shape[0], *matrix_to_csr(A2)[2:])
    assert g1 == g2 and hash(g1) == hash(g2) and g1 != g3
    ops = as_operators([A.toarray(), A.toarray(), A], N=8)
    assert all(isinstance(o, MatrixOperator) for o in ops)
    assert len({o.geom for o in ops}) == 1  # equal matrices: one device context
    assert ops[0].shape == A.shape and ops[0].T.shape == A.shape[::-1] and ops[0].T._adjoint
    rt = RayTransform(ParallelBeamGeometry(8, 12))
    assert as_operators([rt])[0] is rt
    with pytest.raises(ValueError, match="N\\*N"):
        MatrixOperator(np.zeros((3, 10)))


def test_loaders_never_unpickle(tmp_path):
    A = _ref()
    D = A.toarray().astype(np.float32)
    np.save(tmp_path / "a.npy", D)
    assert np.array_equal(load_matrix(str(tmp_path / "a.npy")), D)
    sp.save_npz(tmp_path / "s.npz", A)
    assert abs(load_matrix(str(tmp_path / "s.npz")) - A).max() == 0
    np.save(tmp_path / "stack.npy", np.stack([D, 2 * D]))
    L = load_matrix_list(str(tmp_path / "stack.npy"))
    assert len(L) == 2 and np.array_equal(L[1], 2 * D)
    np.savez(tmp_path / "list.npz", A_0=D, A_1=3 * D)
    L = load_matrix_list(str(tmp_path / "list.npz"))
    assert len(L) == 2 and np.array_equal(L[1], 3 * D)
    np.save(tmp_path / "obj.npy", np.array([D, None], dtype=object), allow_pickle=True)
    with pytest.raises(ValueError):  # object arrays need pickle: refused
        load_matrix(str(tmp_path / "obj.npy"))
    (tmp_path / "A_dense_list.pkl").write_bytes(b"\x80\x04N.")
    with pytest.raises(ValueError, match="pickle"):
        load_matrix_list(str(tmp_path / "A_dense_list.pkl"))


def test_ctx_create_matrix_rejects_bad_csr_before_any_hip_call():
    lib = _lib.load()
    m, n, indptr, indices, values = matrix_to_csr(_ref())
    h = C.c_void_p()
    p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    bad_ptr = indptr.copy()
    bad_ptr[-1] += 1  # indptr[m] != nnz
    rc = lib.admm_ctx_create_matrix(C.byref(h), 8, m, len(indices), p(bad_ptr), p(indices), p(values), 0, 1, 0)
    assert rc == -1 and b"indptr" in lib.admm_last_error()
    bad_idx = indices.copy()
    bad_idx[3] = n  # column out of range
    rc = lib.admm_ctx_create_matrix(C.byref(h), 8, m, len(indices), p(indptr), p(bad_idx), p(values), 0, 1, 0)
    assert rc == -1 and b"column" in lib.admm_last_error()
    rc = lib.admm_ctx_create_matrix(C.byref(h), 1, m, len(indices), p(indptr), p(indices), p(values), 0, 1, 0)
    assert rc == -1
    assert lib.admm_ctx_create_matrix(None, 8, m, 0, None, None, None, 0, 1, 0) == -1
