"""GPU parity at the BASELINE.json configurations.

* C2 (256^2, 8-node ring) and C3 (512^2, 16-node ring): whole ADMM trajectories
  against the float64 CPU oracle (oracle/admm.py with the Joseph CSR matrix; the
  iteration's independent node updates run in parallel processes, oracle/parallel.py).
  C3's two-GPU split is checked by running it as 2 ranks on this GPU (gloo) and
  requiring the 1-rank result bitwise (the RCCL path moves the same bytes).
* C4 (1024^2) and C5 (2048^2, float64 samples, anisotropic TV): the CSR matrix is
  2.4 / 10 GB, so the oracle loop runs its float64 vector algebra around the GPU
  operator A (RayTransform @ x, A.T @ y) -- an operator-level oracle whose projector is
  itself pinned against joseph_matrix at these sizes (test_gpu_fullsize_projector.py)
  -- while the product path runs the fused batch kernels (interleaved samples,
  epilogues, CG / TV updates, fixed-order reductions).  Both forward plans
  (unaligned / ray-aligned) must give bitwise the same run.

Tolerances (north star): images and primal / dual trajectories <= 1e-5 relative
Frobenius with float32 samples, <= 1e-9 with float64 samples.
"""
import os

import networkx as nx
import numpy as np
import pytest
import torch

from admm_hip.data import make_precisions, make_sinograms, shepp_logan
from admm_hip.solver import make_operators
from block_6_admm_loop_ver2 import decentralized_admm
from oracle import admm as oadmm
from oracle.parallel import NodePool

pytestmark = pytest.mark.gpu
ORACLE_THREADS = 8  # the operator-level oracle's node updates in threads (the box's 16-core share)


def rel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def problem(N, V, a_per, dtype="float32"):
    ops = make_operators(N, V, a_per * V, dtype=dtype, device=0)
    ph = shepp_logan(N)
    sinos = make_sinograms(ops, ph, 0.005, seed=1000)
    Wi, Q = make_precisions(ops)
    return ops, ph.numpy(), sinos, Wi, Q


def gpu_run(ops, sinos, G, Wi, Q, N, iters, ph, **kw):
    x, h = decentralized_admm(ops, sinos, G, Wi, Q, N, lam_tv=0.02, rho=2.0, max_iters=iters,
                              eps_pri=0.0, eps_dual=0.0, verbose=False, phantom_true=ph,
                              write_params=False, **kw)
    torch.cuda.synchronize()
    return np.stack(x), h


def check(x, h, xo, ho, tol):
    errs = {"x": rel(x, np.stack(xo)), "primal": rel(h["primal"], ho["primal"]),
            "dual": rel(h["dual"], ho["dual"]), "obj": rel(h["obj_total"], ho["obj_total"]),
            "sb_res": rel(np.stack(h["sb_res_history"]), np.stack(ho["sb_res_history"]))}
    print({k: f"{v:.2e}" for k, v in errs.items()})
    assert errs["x"] < tol and errs["primal"] < tol and errs["dual"] < tol, errs
    assert errs["obj"] < max(10 * tol, 1e-4) and errs["sb_res"] < max(100 * tol, 1e-3), errs


@pytest.mark.timeout(600)
@pytest.mark.parametrize("N,V,iters", [(256, 8, 5), (512, 16, 20)], ids=["C2", "C3"])
def test_ring_trajectory_matches_oracle(cuda, N, V, iters):
    """Whole trajectories at BASELINE sizes: C3 (512^2, 16-node ring) over its full 20 ADMM
    iterations and C2 (256^2, 8-node ring) over 5 (block_6_admm_loop_ver2.py:69-289).
    Besides the whole-history relative errors, every iteration's primal / dual residual and
    objective is compared on its own (float32 sample drift would show as a growing
    per-iteration error).  The oracle's node updates run in oracle/parallel.NodePool: one
    worker per node (the GPU box's 16-core share runs C3's 16 at once), each holding its
    node's state for the whole trajectory, over one memory-mapped Joseph CSR matrix."""
    ops, ph, sinos, Wi, Q = problem(N, V, 96)
    G = nx.cycle_graph(V)
    x, h = gpu_run(ops, sinos, G, Wi, Q, N, iters, ph)
    sin_h = [s.double().cpu().numpy() for s in sinos]
    with NodePool(N, 96, procs=min(V, 16), verbose=True) as pool:
        xo, ho = oadmm.decentralized_admm([pool.A] * V, sin_h, G, Q, N, lam_tv=0.02, rho=2.0,
                                          max_iters=iters, eps_pri=0.0, eps_dual=0.0,
                                          phantom_true=ph, pool=pool)
    assert len(h["primal"]) == len(ho["primal"]) == iters
    check(x, h, xo, ho, 1e-5)
    per_it = {k: max(abs(a - b) / abs(b) for a, b in zip(h[k], ho[k])) for k in ("primal", "dual", "obj_total")}
    print(f"{N}^2 x {iters} iterations, max per-iteration relative error:",
          {k: f"{v:.2e}" for k, v in per_it.items()})
    assert per_it["primal"] < 1e-5 and per_it["dual"] < 1e-5 and per_it["obj_total"] < 1e-4, per_it


def _c3_rank(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ops, ph, sinos, Wi, Q = problem(512, 16, 96)
        x, h = gpu_run(ops, sinos, nx.cycle_graph(16), Wi, Q, 512, 2, ph)
        q.put((rank, x, np.asarray(h["primal"]), np.asarray(h["dual"])))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(400)
def test_c3_two_ranks_match_one_rank_bitwise(cuda):
    """C3 as deployed: 16 nodes split 8 + 8 over two ranks (ring halo exchange)."""
    import socket
    import torch.multiprocessing as mp
    ops, ph, sinos, Wi, Q = problem(512, 16, 96)
    x1, h1 = gpu_run(ops, sinos, nx.cycle_graph(16), Wi, Q, 512, 2, ph)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_c3_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=350) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, x2, pr, du in res:
        assert np.array_equal(x1, x2), rank
        assert np.array_equal(np.asarray(h1["primal"]), pr) and np.array_equal(np.asarray(h1["dual"]), du)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("N,V,dtype,tv,graph,tvi,tol", [
    (1024, 8, "float32", "iso", "ring", 10, 1e-5),        # C4 size (8 of its 32 nodes per GPU)
    (2048, 4, "float64", "aniso", "complete", 4, 1e-9),   # C5 size, precision and TV
], ids=["C4-1024-f32", "C5-2048-f64-aniso"])
def test_large_x_updates_match_operator_oracle(cuda, monkeypatch, N, V, dtype, tv, graph, tvi, tol):
    ops, ph, sinos, Wi, Q = problem(N, V, 96, dtype)
    G = nx.cycle_graph(V) if graph == "ring" else nx.complete_graph(V)
    runs = []
    for plan in ("0", "1", "2", "5"):
        monkeypatch.setenv("ADMM_FWD_PLAN", plan)
        runs.append(gpu_run(ops, sinos, G, Wi, Q, N, 2, ph, tv_kind=tv, tv_iters=tvi))
    monkeypatch.delenv("ADMM_FWD_PLAN")
    for xr, hr in runs[1:]:
        assert np.array_equal(runs[0][0], xr) and runs[0][1]["primal"] == hr["primal"]
    x, h = runs[1]
    sin_h = [s.double().cpu().numpy() for s in sinos]
    xo, ho = oadmm.decentralized_admm(ops, sin_h, G, Q, N, lam_tv=0.02, rho=2.0, max_iters=2,
                                      eps_pri=0.0, eps_dual=0.0, phantom_true=ph, tv_kind=tv,
                                      tv_iters=tvi, threads=ORACLE_THREADS)
    check(x, h, xo, ho, tol)


@pytest.mark.timeout(900)
def test_c5_share_full_inner_count_matches_operator_oracle(cuda):
    """C5's arithmetic at its real inner count: 2048^2, the 8-node
    complete graph of C5's per-GPU share (C5s), float64 samples, anisotropic TV, split-Bregman
    10 x 5, 2 ADMM iterations -- whole histories (every per-node key the reference records,
    block_6_admm_loop_ver2.py:310-326) and images against the operator-level oracle at 1e-9.
    The product path runs z derived from the endpoint images (ABI 7), the oracle the
    reference's literal (a_a + a_b) / 2 -- equal to rounding."""
    N, V = 2048, 8
    ops, ph, sinos, Wi, Q = problem(N, V, 96, "float64")
    G = nx.complete_graph(V)
    x, h = gpu_run(ops, sinos, G, Wi, Q, N, 2, ph, tv_kind="aniso", tv_iters=10, cg_iters=5)
    sin_h = [s.double().cpu().numpy() for s in sinos]
    xo, ho = oadmm.decentralized_admm(ops, sin_h, G, Q, N, lam_tv=0.02, rho=2.0, max_iters=2,
                                      eps_pri=0.0, eps_dual=0.0, phantom_true=ph, tv_kind="aniso",
                                      tv_iters=10, cg_iters=5, threads=ORACLE_THREADS)
    check(x, h, xo, ho, 1e-9)
    for k in ("obj_per_node", "mse_sino_per_node", "img_mse_per_node", "pri_per_node", "dual_per_node"):
        e = rel(np.stack(h[k]), np.stack(ho[k]))
        print(k, f"{e:.2e}")
        assert e < 1e-9, (k, e)
    for k in range(V):
        assert rel(x[k], xo[k]) < 1e-9, k
