"""GPU parity: HIP projector / adjoint / column norms / TV stencils vs the CPU oracle.

Oracle: oracle/geometry.py (Joseph matrix, float64) and oracle/tv.py.
Tolerances (relative Frobenius): float32 samples 2e-6, float64 samples 1e-12.
"""
import math

import numpy as np
import pytest
import torch

from admm_hip.geometry import ParallelBeamGeometry, RayTransform, get_ctx
from admm_hip import _lib
from oracle import tv as otv
from oracle.geometry import Geometry, joseph_matrix, shepp_logan, joseph_adjoint_gather

pytestmark = pytest.mark.gpu

# (N, angles): 45 angles put one midpoint exactly at pi/2 (cos = 6e-17, dl ~ 0);
# 48 and 37 are non-multiples of the 64-wide tiles; 2 is the smallest image; 150 angles take
# the back projector past one 96-angle window chunk.
CASES = [(2, 3), (16, 12), (37, 19), (48, 36), (64, 48), (64, 45), (128, 96), (64, 150)]
TOL = {"float32": 2e-6, "float64": 1e-12}


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / max(np.linalg.norm(np.asarray(b)), 1e-300))


@pytest.mark.parametrize("N,a", CASES)
@pytest.mark.parametrize("dtype", ["float32", "float64"])
def test_forward_matches_oracle(cuda, N, a, dtype):
    A = joseph_matrix(Geometry(N, a))
    op = RayTransform(ParallelBeamGeometry(N, a), dtype)
    rng = np.random.default_rng(N * 100 + a)
    X = rng.standard_normal((3, N * N))
    X[0] = shepp_logan(N, 2).ravel()
    tdt = torch.float64 if dtype == "float64" else torch.float32
    Y = (op @ torch.as_tensor(X, dtype=tdt, device=cuda)).double().cpu().numpy()
    Xs = torch.as_tensor(X, dtype=tdt).double().numpy()  # the values the GPU actually saw
    for v in range(3):
        assert rel(Y[v], A @ Xs[v]) < TOL[dtype], (v, rel(Y[v], A @ Xs[v]))


@pytest.mark.parametrize("N,a", CASES)
@pytest.mark.parametrize("dtype", ["float32", "float64"])
def test_adjoint_matches_oracle(cuda, N, a, dtype):
    A = joseph_matrix(Geometry(N, a))
    op = RayTransform(ParallelBeamGeometry(N, a), dtype)
    rng = np.random.default_rng(7 + N + a)
    Yi = rng.standard_normal((2, A.shape[0]))
    tdt = torch.float64 if dtype == "float64" else torch.float32
    X = (op.T @ torch.as_tensor(Yi, dtype=tdt, device=cuda)).double().cpu().numpy()
    Ys = torch.as_tensor(Yi, dtype=tdt).double().numpy()
    for v in range(2):
        assert rel(X[v], A.T @ Ys[v]) < TOL[dtype]
        assert rel(X[v], joseph_adjoint_gather(Geometry(N, a), Ys[v])) < TOL[dtype]


# N = 2: L = 2/(N max(|cos|, |sin|)) > 1, so the float weights run scaled by 2^-wexp (k_back)
@pytest.mark.parametrize("N,a", [(2, 3), (3, 5), (16, 12), (64, 45), (128, 96)])
def test_column_norms_match_oracle(cuda, N, a):
    A = joseph_matrix(Geometry(N, a))
    W = np.maximum(np.asarray(A.multiply(A).sum(axis=0)).ravel(), 1e-12)
    Wg = RayTransform(ParallelBeamGeometry(N, a)).column_norms_sq()
    assert rel(Wg, W) < 2e-6


def test_numpy_roundtrip_and_batch_of_one(cuda):
    op = RayTransform(ParallelBeamGeometry(32, 20))
    A = joseph_matrix(Geometry(32, 20))
    x = np.random.default_rng(1).standard_normal(32 * 32)
    y = op @ x  # numpy in -> numpy out
    assert isinstance(y, np.ndarray) and y.shape == (20 * 32,)
    assert rel(y, A @ x.astype(np.float32).astype(np.float64)) < 2e-6
    assert (op.T @ y).shape == (32 * 32,)


@pytest.mark.parametrize("dtype", ["float32", "float64"])
def test_detector_wider_than_image(cuda, dtype):
    """det_width_factor > 1 (block_2_load_odl_data.py:16,42): rays outside the image are 0
    (every k_f of the back projector is positive without a bias here)."""
    g = Geometry(40, 30, det_width_factor=1.5)
    A = joseph_matrix(g)
    op = RayTransform(ParallelBeamGeometry(40, 30, det_width_factor=1.5), dtype)
    tdt = torch.float64 if dtype == "float64" else torch.float32
    x = torch.as_tensor(np.random.default_rng(3).standard_normal(1600), dtype=tdt)
    y = torch.as_tensor(np.random.default_rng(4).standard_normal(A.shape[0]), dtype=tdt)
    xs, ys = x.double().numpy(), y.double().numpy()
    assert rel((op @ x.to(cuda)).double().cpu().numpy(), A @ xs) < TOL[dtype]
    assert rel((op.T @ y.to(cuda)).double().cpu().numpy(), A.T @ ys) < TOL[dtype]


def test_finer_detector_rejected(cuda):
    with pytest.raises(_lib.AdmmError):
        RayTransform(ParallelBeamGeometry(32, 10, det_width_factor=0.5)) @ np.zeros(1024)


def test_far_off_detector_rejected_by_the_float_taps_range(cuda):
    """admm_ctx_create refuses a geometry whose bin positions reach 2^20 (the float back
    projector's biased k_f, kernels.hpp kf_split) instead of addressing garbage."""
    import ctypes as C
    lib = _lib.load()
    h = C.c_void_p()
    far = _lib.Geom(32, 10, 32, 0, 0.0, float(np.pi), -2.0e6 - 2.0, -2.0e6)  # k_f ~ 3.2e7
    with pytest.raises(_lib.AdmmError, match="2\\^20"):
        _lib.check(lib.admm_ctx_create(C.byref(h), C.byref(far), _lib.ADMM_DTYPE_F32, 1, 0), "admm_ctx_create")
    ok = _lib.Geom(32, 10, 32, 0, 0.0, float(np.pi), -1.0, 1.0)
    _lib.check(lib.admm_ctx_create(C.byref(h), C.byref(ok), _lib.ADMM_DTYPE_F32, 1, 0), "admm_ctx_create")
    _lib.check(lib.admm_ctx_destroy(h), "admm_ctx_destroy")


@pytest.mark.parametrize("N", [2, 33, 64])
def test_tv_stencils_match_oracle(cuda, N):
    import ctypes as C
    ctx = get_ctx(ParallelBeamGeometry(N, 4), "float64", 0)
    rng = np.random.default_rng(N)
    x = torch.as_tensor(rng.standard_normal((2, N * N)), device=cuda)
    gx = torch.empty_like(x)
    gy = torch.empty_like(x)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(ctx.lib.admm_tv_grad(ctx.h, C.c_void_p(x.data_ptr()), C.c_void_p(gx.data_ptr()),
                                    C.c_void_p(gy.data_ptr()), 2, s), "grad")
    out = torch.empty_like(x)
    _lib.check(ctx.lib.admm_tv_div(ctx.h, C.c_void_p(gx.data_ptr()), C.c_void_p(gy.data_ptr()),
                                   C.c_void_p(out.data_ptr()), 2, s), "div")
    xh = x.cpu().numpy()
    for v in range(2):
        ox, oy = otv.grad(xh[v], N)
        assert np.array_equal(gx[v].cpu().numpy(), ox) and np.array_equal(gy[v].cpu().numpy(), oy)
        assert rel(out[v].cpu().numpy(), otv.div_t(ox, oy, N)) < 1e-14


# ----------------------------------------------------------------------------
# full size (BASELINE: 512^2, 96 angles/node, 8 nodes): size-independent properties
# ----------------------------------------------------------------------------
def test_fullsize_adjointness_linearity_determinism(cuda):
    N, a = 512, 96
    op = RayTransform(ParallelBeamGeometry(N, a))
    g = torch.Generator(device=cuda)
    g.manual_seed(0)
    x = torch.randn((8, N * N), generator=g, device=cuda)
    y = torch.randn((8, a * N), generator=g, device=cuda)
    Ax = op @ x
    Aty = op.T @ y
    lhs = (Ax.double() * y.double()).sum(dim=1)
    rhs = (x.double() * Aty.double()).sum(dim=1)
    assert torch.max(torch.abs(lhs - rhs) / torch.abs(lhs)).item() < 1e-5
    # linearity of the batched projector: A(2x0 - x1) = 2 A x0 - A x1
    comb = op @ (2 * x[0] - x[1])
    assert rel(comb.double().cpu(), (2 * Ax[0].double() - Ax[1].double()).cpu()) < 1e-5
    # determinism (no atomics anywhere): bitwise repeatable
    assert torch.equal(op @ x, Ax)
    assert torch.equal(op.T @ y, Aty)
    # batch of 8 == 8 single projections (node batching does not change results)
    assert torch.equal(op @ x[3], Ax[3])


def test_fullsize_column_norm_point_symmetry(cuda):
    """Rotating the image by pi maps ray (t, k) to (t, N-1-k): W is point symmetric."""
    N = 512
    W = RayTransform(ParallelBeamGeometry(N, 96)).column_norms_sq().reshape(N, N)
    assert np.all(W > 0)
    assert rel(W, W[::-1, ::-1]) < 1e-5


def test_operator_first_use_on_a_side_stream(cuda):
    """A context's scratch is allocated and zero-filled on first use; the zero-fill (null
    stream) must be complete before kernels on a caller's non-blocking stream write the
    scratch (a fresh geometry, so every buffer is allocated inside the stream scope)."""
    N, a = 56, 33
    g = ParallelBeamGeometry(N, a)
    rng = np.random.default_rng(4)
    X = torch.as_tensor(rng.standard_normal((5, N * N)), dtype=torch.float32, device=cuda)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        Y = RayTransform(g, "float32") @ X
        Z = RayTransform(g, "float32").T @ Y
    s.synchronize()
    Yd = RayTransform(g, "float32") @ X
    Zd = RayTransform(g, "float32").T @ Yd
    torch.cuda.synchronize()
    assert torch.equal(Y, Yd) and torch.equal(Z, Zd)
