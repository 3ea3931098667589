"""GPU: operators given as explicit matrices (the reference's A_dense_list,
block_2_load_odl_data.py:68-96 -> block_7_main.py:16-22) drive the same batch path.

admm_ctx_create_matrix keeps A and A^T as device CSR; the x-update, consensus and
statistics kernels run unchanged with the projector replaced by CSR products
(k_csr_fwd / k_back<..., CSR>).  Checked against the float64 oracle with the SAME
matrix (oracle/admm.py takes any scipy matrix), against the matrix-free RayTransform
path on the Joseph matrix it represents, and through the block_5 / block_3 drop-ins.
"""
import networkx as nx
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from admm_hip.data import make_precisions, make_sinograms, shepp_logan
from admm_hip.matrix import MatrixOperator
from admm_hip.solver import make_operators
from block_6_admm_loop_ver2 import decentralized_admm
from oracle import admm as oadmm
from oracle.geometry import Geometry, joseph_matrix

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


@pytest.mark.parametrize("dtype,tol", [("float32", 2e-6), ("float64", 1e-13)])
@pytest.mark.parametrize("kind", ["dense", "csr", "random"])
def test_matrix_operator_products(cuda, dtype, tol, kind):
    N = 24
    A = joseph_matrix(Geometry(N, 30)).tocsr()
    if kind == "random":  # an arbitrary sparse matrix, not a ray transform
        A = sp.random(500, N * N, density=0.05, random_state=3, format="csr")
    op = MatrixOperator(A.toarray() if kind == "dense" else A, dtype=dtype)
    assert op.shape == A.shape
    rng = np.random.default_rng(1)
    X = rng.standard_normal((3, N * N))
    Y = rng.standard_normal((3, A.shape[0]))
    tdt = torch.float64 if dtype == "float64" else torch.float32
    Xs = torch.as_tensor(X, dtype=tdt).double().numpy()
    Ys = torch.as_tensor(Y, dtype=tdt).double().numpy()
    FX = (op @ torch.as_tensor(X, dtype=tdt, device=cuda)).double().cpu().numpy()
    BY = (op.T @ torch.as_tensor(Y, dtype=tdt, device=cuda)).double().cpu().numpy()
    for v in range(3):
        assert rel(FX[v], A @ Xs[v]) < tol
        assert rel(BY[v], A.T @ Ys[v]) < tol
    W = np.maximum(np.asarray(A.multiply(A).sum(axis=0)).ravel(), 1e-12)
    assert rel(op.column_norms_sq(), W) < tol


def _problem(N=32, V=3, dtype="float32"):
    ops = make_operators(N, V, angles_total=96, device=0, dtype=dtype)
    ph = shepp_logan(N)
    sinos = make_sinograms(ops, ph, 0.005)
    A = joseph_matrix(Geometry(N, 96 // V)).tocsr()
    return ops, ph, sinos, A


@pytest.mark.parametrize("dtype,tol", [("float32", 1e-5), ("float64", 1e-9)])
def test_dense_list_admm_matches_oracle(cuda, dtype, tol):
    """decentralized_admm(A_dense_list = the dense Joseph matrices) vs the float64 oracle."""
    N, V = 32, 3
    ops, ph, sinos, A = _problem(N, V, dtype)
    Ad = A.toarray()
    mats = [Ad] * V if dtype == "float32" else [MatrixOperator(Ad, dtype="float64")] * V
    Wi, Q = make_precisions(mats)
    G = nx.cycle_graph(V)
    kw = dict(lam_tv=0.02, rho=2.0, max_iters=4, eps_pri=0.0, eps_dual=0.0)
    x, h = decentralized_admm(mats, sinos, G, Wi, Q, N, verbose=False, phantom_true=ph.numpy(),
                              write_params=False, **kw)
    bo = [s.cpu().numpy().astype(np.float64) for s in sinos]
    xo, ho = oadmm.decentralized_admm([A] * V, bo, G, Q, N, phantom_true=ph.numpy(), **kw)
    assert rel(np.stack(x), np.stack(xo)) < tol
    assert rel(h["primal"], ho["primal"]) < tol
    assert rel(h["dual"], ho["dual"]) < tol
    assert rel(h["mse_sino_total"], ho["mse_sino_total"]) < tol


def test_matrix_path_matches_ray_transform_path(cuda):
    """The CSR products and the matrix-free projector are the same operator: same run."""
    N, V = 32, 4
    ops, ph, sinos, A = _problem(N, V)
    G = nx.cycle_graph(V)
    kw = dict(lam_tv=0.02, rho=2.0, max_iters=4, eps_pri=0.0, eps_dual=0.0, verbose=False,
              write_params=False, phantom_true=ph.numpy())
    Wi, Q = make_precisions(ops)
    x1, h1 = decentralized_admm(ops, sinos, G, Wi, Q, N, **kw)
    mats = [sp.csr_matrix(A)] * V
    Wm, Qm = make_precisions(mats)
    assert rel(np.stack(Wm), np.stack(Wi)) < 2e-6
    x2, h2 = decentralized_admm(mats, sinos, G, Wm, Qm, N, **kw)
    assert rel(np.stack(x2), np.stack(x1)) < 1e-5
    assert rel(h2["primal"], h1["primal"]) < 1e-5


def test_block5_and_block3_dropins_take_matrices(cuda, tmp_path):
    from block_3_graph_and_precisions import build_pixel_connected_Q_provider
    from block_5_node_problem import build_node_problem
    N, V = 32, 3
    ops, ph, sinos, A = _problem(N, V)
    Wi, Q = make_precisions(ops)
    rng = np.random.default_rng(0)
    vs = [ph.numpy().ravel() + 0.02 * rng.standard_normal(N * N) for _ in range(2)]
    qs = [Q(0, 1), Q(0, 2)]
    b = sinos[0].cpu().numpy()
    xr, pr = build_node_problem(ops[0], b, 2.0, vs, N, 0.02, qs)
    pr.solve()
    xm, pm = build_node_problem(A.toarray(), b, 2.0, vs, N, 0.02, qs)
    pm.solve()
    assert rel(xm.value, xr.value) < 1e-5
    assert abs(pm.value - pr.value) <= 1e-5 * abs(pr.value)
    np.save(tmp_path / "A_dense_list.npy", np.stack([A.toarray().astype(np.float32)] * V))
    _, W3, _, keep = build_pixel_connected_Q_provider(str(tmp_path), "A_dense_list.npy", strategy="mst",
                                                      plot_union=False, verbose=False, show_plots=False)
    assert rel(np.stack(W3), np.stack(Wi)) < 2e-6 and tuple(keep.shape) == (V, V, N * N)


def test_matrix_operator_sinograms_and_device_guard(cuda):
    """make_sinograms on matrix operators (MatrixGeometry had no n_angles/n_det)
    returns each node's m rows flat; applying an operator never changes the caller's
    current device (the C entry points restore it)."""
    N = 24
    A = joseph_matrix(Geometry(N, 30)).tocsr()
    op = MatrixOperator(A)
    assert op.geom.n_angles == 1 and op.geom.n_det == A.shape[0]
    ph = shepp_logan(N)
    s = make_sinograms([op], ph, 0.0)[0]
    assert tuple(s.shape) == (A.shape[0],)
    assert rel(s.double().cpu().numpy(), A @ ph.numpy().ravel()) < 2e-6
    before = torch.cuda.current_device()
    for d in range(torch.cuda.device_count()):
        from admm_hip.geometry import ParallelBeamGeometry, RayTransform
        rt = RayTransform(ParallelBeamGeometry(N, 30), "float32", device=d)
        _ = rt @ torch.ones(N * N, device=torch.device("cuda", d))
        _ = rt.T @ torch.ones(30 * N, device=torch.device("cuda", d))
        assert torch.cuda.current_device() == before, (d, before)
