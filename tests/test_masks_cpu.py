"""CPU: per-pixel mask setup -- the host PCG64 replay behind the
chain strategy, C-ABI argument checks (no GPU work), and the oracle's mask structure."""
import ctypes as C

import networkx as nx
import numpy as np
import pytest

from admm_hip import _lib
from admm_hip.masks import chain_orders
from oracle import masks as om


@pytest.mark.parametrize("seed,V,n", [(0, 4, 2000), (3, 16, 3000), (11, 64, 500), (2, 2, 50), (9, 5, 1)])
def test_chain_orders_replay_numpy_stream(seed, V, n):
    """block_3:157,139: rng = default_rng(seed); rng.permutation(V) per pixel, in order."""
    rng = np.random.default_rng(seed)
    ref = np.stack([rng.permutation(V) for _ in range(n)])
    assert np.array_equal(chain_orders(V, n, seed), ref)


def test_chain_orders_state_continuation():
    lib = _lib.load()
    rng = np.random.default_rng(42)
    st = rng.bit_generator.state
    s, inc = st["state"]["state"], st["state"]["inc"]
    m = (1 << 64) - 1
    pcg = (C.c_uint64 * 4)(s >> 64, s & m, inc >> 64, inc & m)
    out = np.empty((7, 6), dtype=np.int32)
    po = (C.c_uint64 * 6)()
    assert lib.admm_chain_orders(pcg, 0, 0, 6, 7, out.ctypes.data_as(C.c_void_p), po) == 0
    for _ in range(7):
        rng.permutation(6)
    st2 = rng.bit_generator.state
    assert (po[0] << 64 | po[1]) == st2["state"]["state"] and po[4] == st2["has_uint32"]
    assert po[5] == st2["uinteger"]


def test_pixel_masks_argument_errors_without_gpu_work():
    lib = _lib.load()
    fake = C.c_void_p(16)  # never dereferenced: validation fails first
    assert lib.admm_pixel_masks(None, 4, 10, 0, 2, 0, None, fake, None) == -1
    assert lib.admm_pixel_masks(fake, 1, 10, 0, 2, 0, None, fake, None) == -1
    assert lib.admm_pixel_masks(fake, 65, 10, 0, 2, 0, None, fake, None) == -1
    assert lib.admm_pixel_masks(fake, 4, 10, 7, 2, 0, None, fake, None) == -1
    assert lib.admm_pixel_masks(fake, 4, 10, _lib.ADMM_MASK_CHAIN, 2, 0, None, fake, None) == -1
    assert b"orders" in lib.admm_last_error()
    assert lib.admm_pixel_masks(fake, 4, 10, 0, 2, 5, None, fake, None) == -1


def _qcol(W, p, qfn_mode="arithmetic"):
    Wi, q = om.precisions(W, qfn_mode)
    V = len(W)
    qc = np.zeros((V, V))
    for i in range(V):
        for j in range(V):
            if i != j:
                qc[i, j] = q(i, j)[p]
    return qc


def test_oracle_mask_structure():
    rng = np.random.default_rng(0)
    V, n = 7, 30
    W = [np.exp(rng.standard_normal(n)) for _ in range(V)]
    _, q = om.precisions(W)
    for strat in ("knn", "mst", "chain"):
        keep = om.build_all_masks(q, V, n, strategy=strat, k=2, seed=1)
        assert np.array_equal(keep, keep.transpose(1, 0, 2))
        assert not keep[np.arange(V), np.arange(V)].any()
        for p in range(n):
            G = nx.from_numpy_array(keep[:, :, p].astype(int))
            assert nx.is_connected(G)
            if strat in ("mst", "chain"):
                assert G.number_of_edges() == V - 1
            if strat == "chain":
                assert max(d for _, d in G.degree()) <= 2
            if strat == "knn":
                assert min(d for _, d in G.degree()) >= 2


def test_oracle_mst_is_maximum_weight_with_kruskal_ties():
    # all-equal weights: Kruskal keeps G.edges() order -> the star around node 0
    qc = np.full((5, 5), 0.5)
    np.fill_diagonal(qc, 0.0)
    m = om.mask_mst(qc, 5)
    assert sorted(map(tuple, np.argwhere(np.triu(m)))) == [(0, 1), (0, 2), (0, 3), (0, 4)]
    # distinct weights: the heaviest tree
    rng = np.random.default_rng(4)
    W = [np.exp(rng.standard_normal(3)) for _ in range(6)]
    qc = _qcol(W, 1)
    m = om.mask_mst(qc, 6)
    best = nx.maximum_spanning_tree(nx.from_numpy_array(qc))
    assert sum(qc[i, j] for i, j in np.argwhere(np.triu(m))) == pytest.approx(
        sum(d["weight"] for _, _, d in best.edges(data=True)))
