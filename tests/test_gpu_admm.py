"""GPU parity of the full decentralized ADMM hot path vs the CPU oracle.

Same inputs on both sides (the GPU-synthesised float32 sinograms, cast to
float64 for the oracle).  North-star tolerance: reconstructed images and the
primal / dual residual trajectories within 1e-5 relative Frobenius of the
float64 oracle (float32 projector samples, float64 solver state).  With float64
samples (the C5 configuration) the bar is 1e-9.
"""
import networkx as nx
import numpy as np
import pytest
import torch

from admm_hip.data import make_precisions, make_sinograms, shepp_logan
from admm_hip.solver import make_operators
from block_5_node_problem import build_node_problem
from block_6_admm_loop_ver2 import decentralized_admm
import block_6_admm_loop
from oracle import admm as oadmm
from oracle import node_solver as ons
from oracle.geometry import Geometry, joseph_matrix

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def setup_problem(N, V, angles_total, dtype="float32", seed=1000):
    ops = make_operators(N, V, angles_total, dtype=dtype, device=0)
    ph = shepp_logan(N)
    sinos = make_sinograms(ops, ph, 0.005, seed=seed)
    Wi, Q = make_precisions(ops)
    A = joseph_matrix(Geometry(N, ops[0].geom.n_angles))
    sin_h = [s.double().cpu().numpy() for s in sinos]
    return ops, ph.numpy(), sinos, Wi, Q, A, sin_h


def node_weights(Wi, seed=5):
    """Per-node, per-pixel distinct W_i (all nodes share one geometry, so the
    make_precisions W_i are identical and weighted fusion would equal the midpoint)."""
    rng = np.random.default_rng(seed)
    W = [np.asarray(w.double().cpu().numpy() if hasattr(w, "cpu") else w, dtype=np.float64)
         * np.exp(0.7 * rng.standard_normal(np.asarray(w.shape).prod())) for w in Wi]
    Q = lambda i, j: np.maximum(0.5 * (W[i] + W[j]), 1e-12)  # noqa: E731  block_3:33-39
    return W, Q


def compare(G, N, V, iters, angles_total, dtype="float32", tol=1e-5, tv_kind="iso", lam=0.02,
            rho=2.0, tv_iters=10, cg_iters=5, fusion="midpoint", g_tol=None):
    ops, ph, sinos, Wi, Q, A, sin_h = setup_problem(N, V, angles_total, dtype)
    Wo = None
    if fusion == "weighted":
        Wi, Q = node_weights(Wi)
        Wo = Wi
    x, h = decentralized_admm(ops, sinos, G, Wi, Q, N, lam_tv=lam, rho=rho, max_iters=iters,
                              eps_pri=0.0, eps_dual=0.0, verbose=False, phantom_true=ph,
                              tv_kind=tv_kind, tv_iters=tv_iters, cg_iters=cg_iters,
                              write_params=False, fusion=fusion)
    xo, ho = oadmm.decentralized_admm([A] * V, sin_h, G, Q, N, lam_tv=lam, rho=rho,
                                      max_iters=iters, eps_pri=0.0, eps_dual=0.0, phantom_true=ph,
                                      tv_kind=tv_kind, tv_iters=tv_iters, cg_iters=cg_iters,
                                      fusion=fusion, Wi_list=Wo)
    assert set(h) >= set(oadmm.HISTORY_KEYS)
    errs = {"x": rel(np.stack(x), np.stack(xo))}
    for k in ("primal", "dual"):
        errs[k] = rel(h[k], ho[k])
    for k in ("obj_total", "mse_sino_total", "img_mse_total"):
        errs[k] = rel(h[k], ho[k])
    errs["g"] = rel(np.stack(h["g_norm_history"]), np.stack(ho["g_norm_history"]))
    print({k: f"{v:.2e}" for k, v in errs.items()})
    assert errs["x"] < tol and errs["primal"] < tol and errs["dual"] < tol, errs
    # diagnostics: same formulas; tolerance covers the float32 A x - b cancellation
    for k in ("obj_total", "mse_sino_total", "img_mse_total"):
        assert errs[k] < max(10 * tol, 1e-4), (k, errs)
    # |g| contains the TV subgradient K^T(Kx/|Kx|), discontinuous where |Kx| ~ 0 (flat
    # phantom regions): image differences of 1e-7 move it by ~1e-5.  Diagnostic only.
    assert errs["g"] < (g_tol or max(20 * tol, 2e-4)), errs  # measured <= 2.4e-5 (C1, 20 iterations)
    return x, h, xo, ho


def test_c1_ring_64_matches_oracle(cuda):
    """BASELINE configs[0]: 64^2 Shepp-Logan, 4-node ring, 20 ADMM iterations."""
    compare(nx.cycle_graph(4), 64, 4, 20, None)


def test_erdos_renyi_matches_oracle(cuda):
    seed = next(s for s in range(100) if nx.is_connected(nx.erdos_renyi_graph(6, 0.5, seed=s)))
    G = nx.erdos_renyi_graph(6, 0.5, seed=seed)
    compare(G, 32, 6, 8, 96)


def test_complete_graph_anisotropic_matches_oracle(cuda):
    compare(nx.complete_graph(5), 32, 5, 6, 100, tv_kind="aniso")


def test_weighted_fusion_matches_oracle(cuda):
    """z = (W_i a_i + W_j a_j)/(W_i + W_j), both endpoint duals."""
    x, h, xo, ho = compare(nx.cycle_graph(4), 48, 4, 10, 192, fusion="weighted")
    # the weighted run differs from the midpoint one (the weights matter)
    xm, hm, _, _ = compare(nx.cycle_graph(4), 48, 4, 10, 192)
    assert rel(h["primal"], hm["primal"]) > 1e-3


def test_weighted_fusion_er_graph_float64(cuda):
    seed = next(s for s in range(100) if nx.is_connected(nx.erdos_renyi_graph(5, 0.6, seed=s)))
    compare(nx.erdos_renyi_graph(5, 0.6, seed=seed), 24, 5, 5, 80, dtype="float64", tol=1e-9,
            fusion="weighted", tv_kind="aniso")


def test_float64_samples_tight(cuda):
    """C5 arithmetic (float64 samples): agreement to 1e-9."""
    compare(nx.cycle_graph(3), 32, 3, 6, 96, dtype="float64", tol=1e-9)


def test_float64_eight_nodes_per_chunk(cuda):
    """float64 samples with V=8 on one device: the 8-wide node chunk (largest LDS windows)."""
    compare(nx.cycle_graph(8), 32, 8, 4, 96, dtype="float64", tol=1e-9)


def test_odd_tv_rounds_and_single_cg(cuda):
    compare(nx.path_graph(3), 24, 3, 4, 72, tv_iters=3, cg_iters=1)


def test_ragged_image_and_node_chunks(cuda):
    """N = 37 (partial 32-pixel tiles everywhere) and V = 11 (one full 8-node chunk and a
    ragged 3-node one) through the whole loop."""
    compare(nx.cycle_graph(11), 37, 11, 4, 11 * 20)


def test_isolated_node_matches_oracle(cuda):
    """A node with no neighbours (deg 0: D = 0, c = 0, its x-update is the TV-regularised
    least-squares problem alone; _ver2:85-97 with an empty neighbour list)."""
    G = nx.path_graph(3)
    G.add_node(3)
    # the isolated node's |g| is its TV subgradient term alone (no consensus pull): 2e-6
    # image differences move it by 3e-4 there (measured), so its diagnostic bar is 1e-3
    compare(G, 32, 4, 4, 96, g_tol=1e-3)


def test_graph_without_edges_matches_oracle(cuda):
    """E = 0: every node independent, residuals identically zero (_ver2:232-289 over no
    edges), statistics table of node rows only."""
    G = nx.empty_graph(3)
    x, h, xo, ho = compare(G, 24, 3, 3, 72)
    assert np.all(np.asarray(h["primal"]) == 0) and np.all(np.asarray(h["dual"]) == 0)


def test_single_node_matches_oracle(cuda):
    compare(nx.empty_graph(1), 32, 1, 3, 48)


def test_cg_steps_beyond_the_direction_ring(cuda):
    """cg_iters = 9 > the 8-slot direction ring: the TV update then folds in only the round's
    last CG step (the F = 1 path of enqueue_update) -- same iteration, same oracle."""
    compare(nx.cycle_graph(4), 32, 4, 3, 96, tv_iters=2, cg_iters=9)


def test_deterministic_bitwise(cuda):
    ops, ph, sinos, Wi, Q, A, _ = setup_problem(48, 4, 96)
    G = nx.cycle_graph(4)
    runs = [decentralized_admm(ops, sinos, G, Wi, Q, 48, lam_tv=0.02, rho=2.0, max_iters=3,
                               verbose=False, write_params=False) for _ in range(2)]
    assert all(np.array_equal(a, b) for a, b in zip(runs[0][0], runs[1][0]))
    assert runs[0][1]["primal"] == runs[1][1]["primal"]


@pytest.mark.parametrize("N,V,angles,dtype", [(96, 8, 384, "float32"), (64, 5, 200, "float64")])
def test_forward_plans_bitwise_equal(cuda, monkeypatch, N, V, angles, dtype):
    """The grouped forward projector's ray layouts (plain 64-ray chunks, rays aligned per
    row segment and angle, chunks aligned per row segment and chunk, each with and without
    rays clipped to the segment -- a clipped ray's partial is an exact 0) and block orders only
    redistribute work: every (segment, ray) partial is
    the same sum in the same order, so whole ADMM runs are bitwise identical."""
    ops, ph, sinos, Wi, Q, A, _ = setup_problem(N, V, angles, dtype)
    G = nx.cycle_graph(V)
    runs = []
    for plan, natural in (("0", "0"), ("1", "0"), ("2", "0"), ("3", "0"), ("4", "0"), ("5", "0"),
                          ("0", "1"), ("2", "1"), ("5", "1")):
        monkeypatch.setenv("ADMM_FWD_PLAN", plan)
        monkeypatch.setenv("ADMM_FWD_NATURAL_ORDER", natural)
        runs.append(decentralized_admm(ops, sinos, G, Wi, Q, N, lam_tv=0.02, rho=2.0, max_iters=2,
                                       verbose=False, write_params=False))
    for x, h in runs[1:]:
        assert all(np.array_equal(a, b) for a, b in zip(runs[0][0], x))
        assert runs[0][1]["primal"] == h["primal"]


def test_stop_criterion_and_ver1_surface(cuda):
    ops, ph, sinos, Wi, Q, A, _ = setup_problem(32, 3, 96)
    x, h = block_6_admm_loop.decentralized_admm(ops, sinos, nx.cycle_graph(3), Wi, Q, 32,
                                                lam_tv=0.02, rho=2.0, max_iters=50,
                                                eps_pri=1e9, eps_dual=1e9, verbose=False,
                                                scs_total_iters=7, scs_chunk_iters=3,
                                                write_params=False)
    assert len(h["primal"]) == 1  # stopped after the first iteration (_ver2:286-289)
    assert h["primal_res"] is h["primal"] and h["obj"] is h["obj_total"]


def test_build_node_problem_matches_oracle(cuda):
    """block_5 surface: one node with two neighbour terms, two warm-started solves."""
    N = 40
    ops, ph, sinos, Wi, Q, A, sin_h = setup_problem(N, 1, 60)
    rng = np.random.default_rng(5)
    vs = [ph.ravel() + 0.05 * rng.standard_normal(N * N) for _ in range(2)]
    qs = [Wi[0] * (1.0 + 0.5 * rng.random(N * N)) for _ in range(2)]
    xi, prob = build_node_problem(ops[0], sinos[0].reshape(-1), 2.0, vs, N, 0.02, qs)
    st = ons.NodeState.zeros(N * N)
    b = sin_h[0].reshape(-1)
    D = qs[0] + qs[1]
    c = qs[0] * vs[0] + qs[1] * vs[1]
    prm = ons.NodeParams(rho=2.0, lam=0.02, mu=0.2)
    for _ in range(2):
        prob.solve(solver="SCS", eps=1e-2, max_iters=50, warm_start=True, verbose=False,
                   acceleration_lookback=20)
        d = ons.node_update(A, A.T @ b, b, D, c, list(zip(qs, vs)), st, N, prm)
        assert rel(xi.value, st.x) < 1e-5
        assert abs(prob.value - d.obj) / abs(d.obj) < 1e-5
    assert prob.solver_stats.num_iters == 50 and prob.status == "optimal_inaccurate"


def test_build_node_problem_cached_in_ver2_loop(cuda):
    """The reference's own loop shape (block_6_admm_loop_ver2.py:81-123, 210-230): a new
    build_node_problem per node per outer iteration, the literal _ver2 edge updates between the
    iterations (oracle.admm.edge_update_literal).  4-node ring at 512^2 (C3's image), 5 outer
    iterations = 20 calls.  The cached batches with warm_start=False give bitwise the uncached
    path; warm_start=True (the reference's keyword) continues each node from its previous
    x-update; a cached call costs at most 2x the x-update it replays."""
    import time
    import block_5_node_problem as b5
    N, V, iters = 512, 4, 5
    ops = make_operators(N, V, 96 * V, dtype="float32", device=0)
    sinos = [s.reshape(-1) for s in make_sinograms(ops, shepp_logan(N), 0.005, seed=1000)]
    Wi, Q = make_precisions(ops)
    G = nx.cycle_graph(V)

    def loop(cache, warm):
        b5.clear_cache()
        b5.CACHE_ENTRIES = 256 if cache else 0
        x = [np.zeros(N * N) for _ in range(V)]
        y = {(min(i, j), max(i, j), k): np.zeros(N * N) for i, j in G.edges() for k in (i, j)}
        z = {(min(i, j), max(i, j)): np.zeros(N * N) for i, j in G.edges()}
        out, t_call, t_upd = [], [], []
        for _ in range(iters):
            new_x = [None] * V
            for i in range(V):
                vs, qs = [], []
                for j in G.neighbors(i):
                    key = (min(i, j), max(i, j))
                    vs.append(z[key] - y[(key[0], key[1], i)])
                    qs.append(Q(i, j))
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                xi, prob = b5.build_node_problem(ops[i], sinos[i], 2.0, vs, N, 0.02, qs)
                prob.solve(solver="SCS", eps=1e-2, max_iters=50, acceleration_lookback=20, verbose=False,
                           warm_start=warm)
                t_call.append(time.perf_counter() - t0)
                new_x[i] = xi.value
                out.append((xi.value.copy(), prob.value))
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                if cache:  # the x-update alone, replayed once more on a scratch copy of the state
                    nb = prob.nb
                    saved = [t.clone() for t in (nb.x_ext, nb.d, nb.e)]
                    ev[0].record()
                    nb.node_update()
                    ev[1].record()
                    torch.cuda.synchronize()
                    t_upd.append(ev[0].elapsed_time(ev[1]) * 1e-3)
                    for t, s in zip((nb.x_ext, nb.d, nb.e), saved):
                        t.copy_(s)
            x = new_x
            z, y = oadmm.edge_update_literal(G, x, y, z)
        return out, t_call, t_upd

    try:
        ref, t_fresh, _ = loop(False, False)
        cold, t_cold, _ = loop(True, False)
        for (xa, va), (xb, vb) in zip(ref, cold):
            assert np.array_equal(xa, xb) and va == vb
        warm, t_warm, t_upd = loop(True, True)
    finally:
        b5.clear_cache()
        b5.CACHE_ENTRIES = 256
    # warm starts: the first iteration's calls are the cold ones; later ones move less
    assert all(np.array_equal(a[0], b[0]) for a, b in zip(ref[:V], warm[:V]))
    call = float(np.median(t_warm[V:]))
    upd = float(np.median(t_upd[V:]))
    print(f"per call: uncached {np.median(t_fresh[V:]) * 1e3:.2f} ms, cached cold {np.median(t_cold[V:]) * 1e3:.2f} ms, "
          f"cached warm {call * 1e3:.2f} ms; one replayed x-update {upd * 1e3:.2f} ms")
    assert call <= 2.0 * upd, (call, upd)


def test_build_node_problem_no_neighbours_no_tv(cuda):
    """test_block5_with_aggregate.py:59-67 shape: rho=0, no neighbours; lam=0 -> least squares."""
    N = 24
    ops, ph, sinos, Wi, Q, A, sin_h = setup_problem(N, 1, 72)
    xi, prob = build_node_problem(ops[0], sinos[0].reshape(-1), 0.0, [], N, 0.0, [])
    prob.solve(max_iters=200)
    b = sin_h[0].reshape(-1)
    r0 = np.linalg.norm(b)
    r1 = np.linalg.norm(A @ xi.value - b)
    assert r1 < 0.1 * r0


def test_pipelined_statistics_equal_per_iteration_readback(cuda):
    """run_admm's pipelined mode (eps = 0: the stop test cannot fire, statistics read back
    once after the loop) gives bitwise the histories and images of the per-iteration
    read-back; with the 5-node unequal-angle split (two batches) as well."""
    from admm_hip.admm import run_admm
    for V, angles in ((4, 96 * 4), (5, 192)):
        ops, ph, sinos, Wi, Q, A, _ = setup_problem(48, V, angles)
        G = nx.cycle_graph(V)
        runs = [run_admm(ops, sinos, G, Wi, Q, 48, lam_tv=0.02, rho=2.0, max_iters=4, eps_pri=0.0,
                         eps_dual=0.0, verbose=False, phantom_true=ph, write_params=False, pipeline=pl)
                for pl in (None, False)]
        (x1, h1), (x2, h2) = runs
        assert all(np.array_equal(a, b) for a, b in zip(x1, x2))
        for k in h1:
            assert np.array_equal(np.asarray(h1[k]), np.asarray(h2[k]), equal_nan=True), k
