"""GPU parity of the per-pixel mask kernel (admm_pixel_masks) and the masked-Q
ADMM path against the oracle restatement of block_3_graph_and_precisions.py:62-187.

Bit-exact for MST (Kruskal's stable tie order is a strict total order) and chain
(the numpy PCG64 stream is replayed).  kNN is bit-exact where the top-k choice
has no ties; on tied weights the reference's pick is np.argpartition's
(unspecified), so tied kNN masks are checked structurally.
"""
import networkx as nx
import numpy as np
import pytest
import torch

from admm_hip.masks import MaskedQProvider, pixel_masks
from block_3_graph_and_precisions import build_pixel_connected_Q_provider
from oracle import masks as om

pytestmark = pytest.mark.gpu


def weights(V, n, kind, seed=0):
    rng = np.random.default_rng(seed)
    if kind == "distinct":
        return [np.exp(rng.standard_normal(n)) for _ in range(V)]
    if kind == "equal":
        w = np.exp(rng.standard_normal(n))
        return [w.copy() for _ in range(V)]
    # a few levels: many ties, some structure
    return [np.exp(rng.integers(0, 3, n).astype(np.float64)) for _ in range(V)]


@pytest.mark.parametrize("strategy", ["mst", "chain", "knn"])
@pytest.mark.parametrize("q_mode", ["arithmetic", "harmonic"])
@pytest.mark.parametrize("V", [3, 6, 17])
def test_masks_match_oracle_tie_free(cuda, strategy, q_mode, V):
    n = 257
    W = weights(V, n, "distinct", seed=V)
    keep = pixel_masks(W, strategy, k=2, seed=5, q_mode=q_mode).cpu().numpy().astype(bool)
    _, q = om.precisions(W, q_mode)
    ref = om.build_all_masks(q, V, n, strategy=strategy, k=2, seed=5)
    assert np.array_equal(keep, ref)


@pytest.mark.parametrize("kind", ["equal", "levels"])
@pytest.mark.parametrize("strategy", ["mst", "chain"])
def test_masks_match_oracle_with_ties(cuda, kind, strategy):
    V, n = 9, 300
    W = weights(V, n, kind, seed=2)
    keep = pixel_masks(W, strategy, seed=3).cpu().numpy().astype(bool)
    _, q = om.precisions(W)
    assert np.array_equal(keep, om.build_all_masks(q, V, n, strategy=strategy, seed=3))


@pytest.mark.parametrize("k", [1, 2, 4])
def test_knn_structure_on_tied_weights(cuda, k):
    V, n = 8, 200
    W = weights(V, n, "levels", seed=1)
    keep = pixel_masks(W, "knn", k=k).cpu().numpy().astype(bool)
    _, q = om.precisions(W)
    for p in range(n):
        m = keep[:, :, p]
        assert np.array_equal(m, m.T) and not m.diagonal().any()
        G = nx.from_numpy_array(m.astype(int))
        assert nx.is_connected(G)
        qc = np.array([[q(i, j)[p] if i != j else -np.inf for j in range(V)] for i in range(V)])
        for i in range(V):
            # node i's own k picks are among its k largest weights (any tie order)
            kth = np.sort(qc[i])[-k]
            assert (qc[i][m[i]] >= kth).sum() >= k


def test_masks_64_nodes_mst(cuda):
    V, n = 64, 24
    W = weights(V, n, "distinct", seed=9)
    keep = pixel_masks(W, "mst").cpu().numpy().astype(bool)
    _, q = om.precisions(W)
    assert np.array_equal(keep, om.build_all_masks(q, V, n, strategy="mst"))


def test_masked_admm_matches_oracle(cuda):
    """Masked precisions through the full hot path (kNN masks, tie-free W)."""
    from test_gpu_admm import rel, setup_problem, node_weights
    from block_6_admm_loop_ver2 import decentralized_admm
    from oracle import admm as oadmm
    N, V = 32, 5
    ops, ph, sinos, Wi, Q, A, sin_h = setup_problem(N, V, 100)
    W, _ = node_weights(Wi, seed=3)
    G = nx.cycle_graph(V)
    _, Wl, Qm, keep = build_pixel_connected_Q_provider(strategy="knn", k=1, Wi_list=W, plot_union=False,
                                                       verbose=False)
    assert isinstance(Qm, MaskedQProvider)
    _, qo = om.precisions(W)
    Qo = om.masked_q(qo, om.build_all_masks(qo, V, N * N, strategy="knn", k=1), N * N)
    assert np.array_equal(Qm(0, 1).cpu().numpy(), Qo(0, 1))
    x, h = decentralized_admm(ops, sinos, G, Wl, Qm, N, lam_tv=0.02, rho=2.0, max_iters=6,
                              eps_pri=0.0, eps_dual=0.0, verbose=False, write_params=False)
    xo, ho = oadmm.decentralized_admm([A] * V, sin_h, G, Qo, N, lam_tv=0.02, rho=2.0, max_iters=6,
                                      eps_pri=0.0, eps_dual=0.0)
    assert rel(np.stack(x), np.stack(xo)) < 1e-5
    assert rel(h["primal"], ho["primal"]) < 1e-5 and rel(h["dual"], ho["dual"]) < 1e-5


def test_dropin_requires_operators_not_pickles(cuda):
    with pytest.raises(FileNotFoundError, match="ops="):
        build_pixel_connected_Q_provider(plot_union=False)
