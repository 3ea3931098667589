"""GPU: the derived consensus (ABI 7) -- midpoint fusion with z never stored.

z_ij is the midpoint of the endpoint images of the last consensus (the single-y invariant,
block_6_admm_loop_ver2.py:210-230 with y_ij,i + y_ij,j = 0), so the library keeps one x_prev
row per x_ext row instead of one z per edge.  Checked here:

* the derived path against the stored-z path (``NodeBatch(derive_z=False)``: z kept per
  edge, the reference's literal (a_a + a_b) / 2) on the same problem: equal to rounding;
* after every consensus z (as every kernel forms it) is exactly (x_a + x_b) / 2 of the
  current images and y = y_old + x_a - z;
* the LDS-tiled consensus kernel (x_ext rows <= 128) and the direct one (more rows) give
  bitwise the same run: a 130-node ring as one rank (130 rows: direct) and as 2 gloo ranks on
  this GPU (65 + 2 halo rows: LDS tile) must agree bit for bit.
"""
import os
import socket

import networkx as nx
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _paths():
    import sys
    for p in (os.path.join(ROOT, "distributed-inverse-problem-admm_amd"), ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)


def _problem(N, V, a_per=24, dtype="float32"):
    _paths()
    from admm_hip.data import make_precisions, make_sinograms, shepp_logan
    from admm_hip.solver import make_operators
    ops = make_operators(N, V, a_per * V, dtype=dtype, device=0)
    ph = shepp_logan(N)
    sinos = make_sinograms(ops, ph, 0.005, seed=1000)
    Wi, Q = make_precisions(ops)
    return ops, ph, sinos, Wi, Q


@pytest.mark.parametrize("dtype", ["float32", "float64"])
def test_derived_z_equals_stored_z(cuda, dtype):
    from admm_hip.plan import make_plan
    from admm_hip.solver import NodeBatch
    N, V = 48, 5
    ops, ph, sinos, Wi, Q = _problem(N, V, dtype=dtype)
    G = nx.complete_graph(V)
    plan = make_plan(G, V)
    runs = {}
    for derive in (True, False):
        nb = NodeBatch(ops[0].geom, dtype, plan, sinos, Q, 2.0, 0.02, 0.2, 3, 4, "iso", ph, 0, derive_z=derive)
        assert (nb.z is None) == derive and (nb.x_prev is None) != derive
        hist = []
        for _ in range(4):
            y_old = nb.y.clone()
            nb.node_update()
            nb.consensus()
            torch.cuda.synchronize()
            hist.append(nb.edge_stats[: len(plan.stored_edges)].cpu().numpy().copy())
            if derive:
                x = nb.x_ext
                for k in range(len(plan.stored_edges)):
                    xa, xb = x[plan.edge_a_row[k]], x[plan.edge_b_row[k]]
                    z = nb.z_of(k)
                    assert torch.equal(z, (xa + xb) * 0.5)
                    assert torch.equal(nb.y[k], y_old[k] + xa - z)
        runs[derive] = (nb.x_ext[:V].cpu().numpy().copy(), np.stack(hist), nb.node_stats.cpu().numpy().copy())
    (xd, hd, nd), (xs, hs, ns) = runs[True], runs[False]
    assert np.linalg.norm(xd - xs) / np.linalg.norm(xs) < 1e-12
    # edge statistics: r = x - z is a difference of nearly equal images, so rounding of z
    # shows relative to |r|, not |x| (still far below the 1e-5 / 1e-9 parity bars)
    assert np.linalg.norm(hd - hs) / np.linalg.norm(hs) < 1e-9
    assert np.linalg.norm(nd - ns) / np.linalg.norm(ns) < 1e-9


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ring_run(V, world=1, rank=0, port=None, q=None):
    import torch.distributed as dist
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ops, ph, sinos, Wi, Q = _problem(24, V, a_per=2)
        from block_6_admm_loop_ver2 import decentralized_admm
        x, h = decentralized_admm(ops, sinos, nx.cycle_graph(V), Wi, Q, 24, lam_tv=0.02, rho=2.0, max_iters=3,
                                  eps_pri=0.0, eps_dual=0.0, verbose=False, phantom_true=ph, write_params=False,
                                  tv_iters=2, cg_iters=2)
        out = (np.stack(x), np.asarray(h["primal"]), np.asarray(h["dual"]))
        if q is not None:
            q.put((rank, out))
        return out
    finally:
        if world > 1:
            dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_lds_and_direct_consensus_kernels_agree_bitwise(cuda, monkeypatch):
    import torch.multiprocessing as mp
    V = 130  # one rank: 130 x_ext rows (> 128: direct kernel); two ranks: 65 + 2 (LDS tile)
    monkeypatch.setenv("ADMM_EDGE_STATE", "derived")  # (stored z is the default wherever it fits)
    x1, p1, d1 = _ring_run(V)
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ring_run, args=(V, 2, r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=250) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, (x2, p2, d2) in res:
        assert np.array_equal(x1, x2), rank
        assert np.array_equal(p1, p2) and np.array_equal(d1, d2), rank


def test_concurrent_batch_streams_bitwise(cuda):
    """RankGroups(streams=2): a rank's 16 nodes as two 8-node batches whose x-updates and edge
    updates run concurrently on two streams -- bitwise the one-batch run (images, every
    history key)."""
    from admm_hip.admm import run_admm
    N, V = 64, 16
    ops, ph, sinos, Wi, Q = _problem(N, V, a_per=12)
    G = nx.cycle_graph(V)
    out = {}
    for st in (1, 2):
        seen = {}
        x, h = run_admm(ops, sinos, G, Wi, Q, N, lam_tv=0.02, rho=2.0, max_iters=3, eps_pri=0.0, eps_dual=0.0,
                        verbose=False, phantom_true=ph, write_params=False, tv_iters=3, cg_iters=3, streams=st,
                        inspect=lambda rg: seen.update(batches=len(rg.batches), streams=rg.streams))
        out[st] = (np.stack(x), h, seen)
    assert out[1][2]["batches"] == 1 and out[2][2]["batches"] == 2 and len(out[2][2]["streams"]) == 2
    assert np.array_equal(out[1][0], out[2][0])
    for k, v in out[1][1].items():
        assert np.array_equal(np.asarray(v), np.asarray(out[2][1][k]), equal_nan=True), k
