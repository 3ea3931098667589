"""CPU: the oracle against the physical pin, its golden vectors and the reference's
algebra (no GPU).  Reference citations are in oracle/*.py."""
import os

import networkx as nx
import numpy as np
import pytest

from oracle import admm as oadmm
from oracle import node_solver as ons
from oracle import tv as otv
from oracle.geometry import (Geometry, default_angles_total, ellipse_phantom, ellipse_radon,
                             joseph_adjoint_gather, joseph_matrix, shepp_logan, shepp_logan_radon,
                             split_angles)

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "oracle_golden.npz"))


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / np.linalg.norm(np.asarray(b)))


# ---------------- geometry (block_2_load_odl_data.py:16-65) ----------------
def test_angle_split_and_defaults():
    assert default_angles_total(64) == 192 and default_angles_total(32) == 180
    assert split_angles(192, 5) == [39, 39, 38, 38, 38]
    assert sum(split_angles(1536, 16)) == 1536


def test_projector_converges_to_analytic_radon():
    """Pins the ODL convention: first-order convergence to the exact line integrals."""
    errs = []
    for N in (32, 64, 128):
        g = Geometry(N, 48)
        errs.append(rel(joseph_matrix(g) @ shepp_logan(N, 4).ravel(), shepp_logan_radon(g).ravel()))
    assert errs[0] > errs[1] > errs[2]
    assert errs[2] < 0.03 and errs[1] / errs[2] > 1.6


def test_wrong_conventions_do_not_match():
    """An off-centre, rotated ellipse: transposed axes, reversed angles or a flipped
    detector give O(1) errors, the ODL convention matches to discretisation error."""
    N = 64
    g = Geometry(N, 48)
    A = joseph_matrix(g)
    table = [[1.0, 0.25, 0.1, 0.45, -0.2, 30.0]]
    ph = ellipse_phantom(N, table, 4)
    ref = ellipse_radon(g, table)
    y = (A @ ph.ravel()).reshape(48, N)
    good = rel(y, ref)
    assert good < 0.08  # O(h) discretisation error of a small ellipse at N=64
    assert rel((A @ ph.T.ravel()).reshape(48, N), ref) > 0.5
    assert rel(y[::-1], ref) > 0.5
    assert rel(y[:, ::-1], ref) > 0.5


def test_gather_adjoint_equals_transpose():
    for N, a in ((16, 12), (33, 17), (40, 45)):
        g = Geometry(N, a)
        A = joseph_matrix(g)
        y = np.random.default_rng(N).standard_normal(A.shape[0])
        assert rel(joseph_adjoint_gather(g, y), A.T @ y) < 1e-13


def test_row_weights_are_joseph():
    """Every ray step distributes exactly L = h/|alpha| over <= 2 pixels."""
    g = Geometry(32, 10)
    A = joseph_matrix(g)
    assert A.shape == (320, 1024)
    row_nnz = np.diff(A.indptr)
    assert row_nnz.max() <= 2 * 32
    th = g.angles
    L = g.h / np.maximum(np.abs(np.cos(th)), np.abs(np.sin(th)))
    # central ray of each angle crosses the full grid: its row sums to N * L
    for t in range(10):
        s = A[t * 32 + 15].sum() + A[t * 32 + 16].sum()
        assert abs(s / 2 - 32 * L[t]) < 0.05 * 32 * L[t]


def test_golden_projector():
    A = joseph_matrix(Geometry(16, 12))
    assert rel(A @ GOLD["proj_x0"], GOLD["proj_Ax0"]) < 1e-14
    assert rel(A.T @ GOLD["proj_y0"], GOLD["proj_ATy0"]) < 1e-14
    W = np.maximum(np.asarray(A.multiply(A).sum(axis=0)).ravel(), 1e-12)
    assert rel(W, GOLD["proj_W"]) < 1e-14
    assert rel(GOLD["radon64_joseph"], GOLD["radon64_analytic"]) < 0.07


# ---------------- TV (block_4_tv_helpers.py:17-46) ----------------
def test_tv_adjoint_and_golden():
    x = GOLD["tv_x"]
    gx, gy = otv.grad(x, 16)
    assert np.array_equal(gx, GOLD["tv_gx"]) and np.array_equal(gy, GOLD["tv_gy"])
    assert rel(otv.div_t(gx, gy, 16), GOLD["tv_div"]) < 1e-15
    assert rel(otv.subgrad(x, 16, "iso"), GOLD["tv_sub_iso"]) < 1e-15
    assert rel(otv.subgrad(x, 16, "aniso"), GOLD["tv_sub_aniso"]) < 1e-15
    rng = np.random.default_rng(0)
    for N in (1, 2, 7, 16):
        x = rng.standard_normal(N * N)
        px, py = rng.standard_normal(N * N), rng.standard_normal(N * N)
        gx, gy = otv.grad(x, N)
        lhs = gx @ px + gy @ py
        assert abs(lhs - x @ otv.div_t(px, py, N)) < 1e-10 * max(1.0, abs(lhs))


def test_grad_matches_reference_forward_differences():
    """block_4_tv_helpers.py:17-23 with C-order X: gx[r,:] = X[r+1,:]-X[r,:], gx[N-1,:]=0."""
    gx, gy = otv.grad(np.arange(9.0) ** 2, 3)
    Xs = (np.arange(9.0) ** 2).reshape(3, 3)
    ex = np.zeros((3, 3))
    ey = np.zeros((3, 3))
    ex[:-1] = Xs[1:] - Xs[:-1]
    ey[:, :-1] = Xs[:, 1:] - Xs[:, :-1]
    assert np.array_equal(gx.reshape(3, 3), ex) and np.array_equal(gy.reshape(3, 3), ey)


def test_reference_div_backward_defect_is_documented():
    """The reference's _div_backward (block_4:25-35) is not the adjoint at the boundary;
    ours is.  Restate the reference formula and show the boundary sign error."""
    N = 5
    rng = np.random.default_rng(1)
    px, py = rng.standard_normal((N, N)), rng.standard_normal((N, N))
    div = np.zeros((N, N))
    div[0, :] -= px[0, :]
    div[1:-1, :] += px[1:-1, :] - px[:-2, :]
    div[-1, :] += px[-2, :]
    div[:, 0] -= py[:, 0]
    div[:, 1:-1] += py[:, 1:-1] - py[:, :-2]
    div[:, -1] += py[:, -2]
    ref = (-div).ravel()
    ours = otv.div_t(px.ravel(), py.ravel(), N)
    inner = np.zeros((N, N), bool)
    inner[1:-1, 1:-1] = True
    assert np.allclose(ref.reshape(N, N)[inner], ours.reshape(N, N)[inner])
    assert not np.allclose(ref, ours)


def test_shrink():
    ux, uy = np.array([3.0, 0.1, 0.0, -4.0]), np.array([4.0, 0.0, 0.0, 3.0])
    dx, dy = otv.shrink(ux, uy, 1.0, "iso")
    assert np.allclose(np.hypot(dx, dy), [4.0, 0.0, 0.0, 4.0])
    assert np.allclose(dx[0] / dy[0], 0.75)
    ax, ay = otv.shrink(ux, uy, 1.0, "aniso")
    assert np.allclose(ax, [2.0, 0.0, 0.0, -3.0]) and np.allclose(ay, [3.0, 0.0, 0.0, 2.0])
    assert np.allclose(otv.shrink(*otv.shrink(ux, uy, 0.0), 0.0), (ux, uy))


# ---------------- node solve (block_5_node_problem.py:6-32) ----------------
def test_node_update_golden_and_descent():
    A = joseph_matrix(Geometry(16, 12))
    b = GOLD["node_b"]
    W = GOLD["proj_W"]
    q1, q2 = W, 1.5 * W
    ph = shepp_logan(16, 4).ravel()
    v1, v2 = ph + 0.01, ph - 0.02
    st = ons.NodeState.zeros(256)
    prm = ons.NodeParams(rho=2.0, lam=0.02, mu=0.2, tv_iters=4, cg_iters=3)
    d = ons.node_update(A, A.T @ b, b, q1 + q2, q1 * v1 + q2 * v2, [(q1, v1), (q2, v2)], st, 16, prm)
    assert rel(st.x, GOLD["node_x"]) < 1e-13
    assert rel([d.obj, d.mse_sino, d.g_norm, d.tv, d.quad], GOLD["node_obj"]) < 1e-12
    f0 = ons.objective(A, b, np.zeros(256), 16, 2.0, 0.02, [(q1, v1), (q2, v2)])
    f1 = ons.objective(A, b, st.x, 16, 2.0, 0.02, [(q1, v1), (q2, v2)])
    assert abs(f1 - d.obj) < 1e-10 * abs(f1) and f1 < f0
    # more iterations keep descending toward the minimiser
    d2 = ons.node_update(A, A.T @ b, b, q1 + q2, q1 * v1 + q2 * v2, [(q1, v1), (q2, v2)], st, 16, prm)
    assert d2.obj <= d.obj * (1 + 1e-12)


def test_cg_identity_matches_plain_cg():
    """Without TV (mu tiny, lam 0) the split-Bregman solver is CG on A^TA + rho D."""
    A = joseph_matrix(Geometry(12, 9))
    rng = np.random.default_rng(3)
    b = rng.standard_normal(A.shape[0])
    D = 1.0 + rng.random(144)
    st = ons.NodeState.zeros(144)
    ons.node_update(A, A.T @ b, b, D, np.zeros(144), [], st, 12,
                    ons.NodeParams(rho=1.0, lam=0.0, mu=1e-14, tv_iters=1, cg_iters=144))
    H = (A.T @ A).toarray() + np.diag(D)
    xs = np.linalg.solve(H, A.T @ b)
    assert rel(st.x, xs) < 1e-6


# ---------------- ADMM loop (block_6_admm_loop_ver2.py) ----------------
def test_admm_golden_trajectory():
    A = joseph_matrix(Geometry(16, 12))
    W = GOLD["proj_W"]
    sinos = list(GOLD["admm_sinos"])
    x, h = oadmm.decentralized_admm([A] * 3, sinos, nx.cycle_graph(3), lambda i, j: W, 16, lam_tv=0.02,
                                    rho=2.0, max_iters=4, eps_pri=0.0, eps_dual=0.0,
                                    phantom_true=shepp_logan(16, 4), tv_iters=4, cg_iters=3)
    assert rel(np.stack(x), GOLD["admm_x"]) < 1e-12
    for k in ("primal", "dual", "obj_total", "mse_sino_total", "img_mse_total"):
        assert rel(h[k], GOLD[f"admm_{k}"]) < 1e-10, k
    assert set(h) == set(oadmm.HISTORY_KEYS) | set(oadmm.EXTRA_KEYS)


def test_node_pool_equals_sequential_loop():
    """oracle/parallel.NodePool (nodes pinned to 2 workers, memory-mapped CSR) and the threaded
    node updates give the sequential loop's trajectory bitwise -- the harnesses of the C2/C3
    GPU trajectory tests and of the operator-level (C4/C5-size) ones."""
    from oracle.parallel import NodePool
    N, V = 16, 5
    A = joseph_matrix(Geometry(N, 12))
    rng = np.random.default_rng(4)
    sinos = [A @ shepp_logan(N, 4).reshape(-1) + 0.01 * rng.standard_normal(A.shape[0]) for _ in range(V)]
    Q = {(i, j): rng.uniform(0.5, 1.5, N * N) for i in range(V) for j in range(V)}
    kw = dict(lam_tv=0.02, rho=2.0, max_iters=3, eps_pri=0.0, eps_dual=0.0, phantom_true=shepp_logan(N, 4),
              tv_iters=3, cg_iters=2)
    G = nx.cycle_graph(V)
    G.add_edge(0, 2)
    x1, h1 = oadmm.decentralized_admm([A] * V, sinos, G, lambda i, j: Q[i, j], N, **kw)
    with NodePool(N, 12, procs=2) as pool:
        x2, h2 = oadmm.decentralized_admm([pool.A] * V, sinos, G, lambda i, j: Q[i, j], N, pool=pool, **kw)
    # the operator-level oracle's threaded node updates (products serialized)
    x3, h3 = oadmm.decentralized_admm([A] * V, sinos, G, lambda i, j: Q[i, j], N, threads=3, **kw)
    for xo, ho in ((x2, h2), (x3, h3)):
        assert np.array_equal(np.stack(x1), np.stack(xo))
        for k in h1:
            assert np.array_equal(np.asarray(h1[k]), np.asarray(ho[k]), equal_nan=True), k


def test_single_y_form_equals_reference_two_dual_form():
    """The device's single-y edge state reproduces _ver2:210-230 literally."""
    rng = np.random.default_rng(9)
    G = nx.Graph([(0, 1), (2, 1), (2, 0), (3, 2)])  # edges listed in non-canonical orientation
    n = 50
    y_lit = {}
    for i, j in G.edges():
        key = (min(i, j), max(i, j))
        y_lit[(key[0], key[1], i)] = np.zeros(n)
        y_lit[(key[0], key[1], j)] = np.zeros(n)
    z_lit = {(min(i, j), max(i, j)): np.zeros(n) for i, j in G.edges()}
    y1 = {e: np.zeros(n) for e in z_lit}
    z1 = {e: np.zeros(n) for e in z_lit}
    for _ in range(5):
        x = [rng.standard_normal(n) for _ in range(4)]
        z_lit, y_lit = oadmm.edge_update_literal(G, x, y_lit, z_lit)
        for (a, b) in oadmm.canonical_edges(G):
            e = (a, b)
            aa, ab = x[a] + y1[e], x[b] - y1[e]
            zn = (aa + ab) * 0.5
            y1[e] = y1[e] + x[a] - zn
            z1[e] = zn
        for e in z_lit:
            assert np.allclose(z_lit[e], z1[e], rtol=0, atol=1e-13)
            assert np.allclose(y_lit[(e[0], e[1], e[0])], y1[e], rtol=0, atol=1e-13)
            # invariant y_ij,i + y_ij,j = 0
            assert np.allclose(y_lit[(e[0], e[1], e[0])] + y_lit[(e[0], e[1], e[1])], 0, atol=1e-13)
            assert np.allclose(z1[e], 0.5 * (x[e[0]] + x[e[1]]), atol=1e-13)


def test_weighted_two_dual_form_equals_reference_weighted_form():
    """Weighted fusion (commented form _ver2:221-222): the oracle's (y, y2) edge state
    reproduces the literal two-dual dict update; y_ij,i + y_ij,j = 0 no longer holds."""
    rng = np.random.default_rng(11)
    G = nx.Graph([(0, 1), (2, 1), (2, 0), (3, 2)])
    n = 40
    W = [np.exp(rng.standard_normal(n)) for _ in range(4)]
    y_lit = {}
    for i, j in G.edges():
        key = (min(i, j), max(i, j))
        y_lit[(key[0], key[1], i)] = np.zeros(n)
        y_lit[(key[0], key[1], j)] = np.zeros(n)
    z_lit = {(min(i, j), max(i, j)): np.zeros(n) for i, j in G.edges()}
    y1 = {e: np.zeros(n) for e in z_lit}
    y2 = {e: np.zeros(n) for e in z_lit}
    for _ in range(4):
        x = [rng.standard_normal(n) for _ in range(4)]
        z_lit, y_lit = oadmm.edge_update_literal(G, x, y_lit, z_lit, Wi_list=W)
        for (a, b) in oadmm.canonical_edges(G):
            e = (a, b)
            aa, ab = x[a] + y1[e], x[b] + y2[e]
            zn = (W[a] * aa + W[b] * ab) / (W[a] + W[b])
            y1[e] = y1[e] + x[a] - zn
            y2[e] = y2[e] + x[b] - zn
            assert np.array_equal(zn, z_lit[e])  # IEEE + is commutative: orientation-free
            assert np.array_equal(y1[e], y_lit[(a, b, a)]) and np.array_equal(y2[e], y_lit[(a, b, b)])
    e = (0, 1)
    assert np.abs(y1[e] + y2[e]).max() > 1e-3


def test_weighted_fusion_with_equal_weights_is_midpoint():
    A = joseph_matrix(Geometry(10, 8))
    W = np.maximum(np.asarray(A.multiply(A).sum(axis=0)).ravel(), 1e-12)
    ph = shepp_logan(10, 2).ravel()
    sinos = [A @ ph + 0.01 * np.random.default_rng(i).standard_normal(A.shape[0]) for i in range(3)]
    kw = dict(lam_tv=0.02, rho=2.0, max_iters=3, eps_pri=0.0, eps_dual=0.0, tv_iters=2, cg_iters=2)
    G = nx.cycle_graph(3)
    xm, hm = oadmm.decentralized_admm([A] * 3, sinos, G, lambda i, j: W, 10, **kw)
    xw, hw = oadmm.decentralized_admm([A] * 3, sinos, G, lambda i, j: W, 10, fusion="weighted",
                                      Wi_list=[W] * 3, **kw)
    assert rel(np.stack(xw), np.stack(xm)) < 1e-13
    assert np.allclose(hw["primal"], hm["primal"], rtol=1e-12)
    with pytest.raises(ValueError):
        oadmm.decentralized_admm([A] * 3, sinos, G, lambda i, j: W, 10, fusion="weighted", **kw)


def test_eps_target_and_stop_rule():
    assert oadmm.eps_target(0) == 2.0
    assert abs(oadmm.eps_target(9) - 2.0 / 10 ** 1.005) < 1e-15
    A = joseph_matrix(Geometry(8, 6))
    W = np.maximum(np.asarray(A.multiply(A).sum(axis=0)).ravel(), 1e-12)
    sinos = [np.ones(A.shape[0]) for _ in range(2)]
    x, h = oadmm.decentralized_admm([A] * 2, sinos, nx.path_graph(2), lambda i, j: W, 8, lam_tv=0.01,
                                    rho=1.0, max_iters=20, eps_pri=1e9, eps_dual=1e9, tv_iters=1,
                                    cg_iters=1)
    assert len(h["primal"]) == 1
    assert np.isnan(h["img_mse_total"][0])  # phantom_true=None (the reference crashes, _ver2:205)


def test_mirror_symmetry_of_the_joseph_operator():
    """The identity the mirror-mode forward projector rests on (kernels.hpp k_fwdg MIRROR):
    with angles (t + 1/2) pi / a over [0, pi) and the symmetric detector of
    block_2_load_odl_data.py:51-52, angle a-1-t (= pi - theta_t) projects image I exactly as
    angle t projects flipud(I), bin for bin (to float64 rounding of the geometry)."""
    import numpy as np
    from oracle.geometry import Geometry, joseph_matrix
    for N, a in ((32, 16), (33, 12), (40, 96)):
        A = joseph_matrix(Geometry(N, a))
        rng = np.random.default_rng(N)
        X = rng.standard_normal((N, N))
        s = (A @ X.ravel()).reshape(a, N)
        sf = (A @ X[::-1, :].ravel()).reshape(a, N)
        t = np.arange(a // 2)
        assert np.abs(sf[t] - s[a - 1 - t]).max() <= 1e-12 * np.abs(s).max()


def test_mirror_identity_of_the_adjoint():
    """The mirror-mode back projector's identity (kernels.hpp k_back_mirror): with A_h the
    first a/2 angles, A^T s = A_h^T s[:a/2] + flipud(A_h^T s_m), s_m[t] = s[a-1-t] -- the real
    A^T s at (i, j) is the half-angle back projection at (i, j) plus the mirrored half's at
    (N-1-i, j)."""
    import numpy as np
    from oracle.geometry import Geometry, joseph_matrix
    for N, a in ((32, 16), (33, 12)):
        A = joseph_matrix(Geometry(N, a))
        Ah = joseph_matrix(Geometry(N, a), angles=list(range(a // 2)))
        rng = np.random.default_rng(a)
        s = rng.standard_normal((a, N))
        full = (A.T @ s.ravel()).reshape(N, N)
        first = (Ah.T @ s[: a // 2].ravel()).reshape(N, N)
        second = (Ah.T @ s[::-1][: a // 2].ravel()).reshape(N, N)[::-1, :]
        assert np.abs(full - (first + second)).max() <= 1e-12 * np.abs(full).max()
