"""Decentralized edge-split ADMM loop on MI355X (the reference's block_6 hot path).

``run_admm`` implements /root/reference/block_6_admm_loop_ver2.py:15-326 with
the node solves and edge updates on the GPU:

  for k in range(max_iters):                         (:69)
      x-update of every local node   -> NodeBatch.node_update   (:81-187)
      halo exchange of x_j           -> HaloExchange.run (RCCL)
      z/y update + residual partials -> NodeBatch.consensus     (:210-253)
      statistics -> history, stop test                          (:189-206,255-289)

Histories carry the reference's keys (:310-326), plus ``sb_res_history`` (the
split-Bregman stationarity residual ||A^T(Ax-b) + rho(Dx-c) + mu K^T e|| of each
accepted x) and ``inner_updates_history`` (x-updates spent per node).

Inner-solve control (row a5).  Default (``inner_tol=None``): one fixed-count x-update
(tv_iters x cg_iters) per node per iteration, deterministic; ``eps_used_history`` is NaN
because no tolerance is applied.  ``inner_tol="reference"``: the accept / tighten loop of
:100-176 -- the node is solved to eps_try = min(1e-2, eps_target(k)) (repeated warm
x-updates until its split-Bregman residual <= eps_try, at most ``max_inner_updates`` per
solve, standing in for SCS's tolerance), accepted if the reference's ||g|| <= eps_target,
else eps_try /= 5 and re-solved, at most twice, then force-accepted; eps_used is the
eps_try of the accepted iterate.  Other nodes' state is untouched while one node
re-solves (masked batch updates).  Nodes may have different operators (the reference's
own angle split gives unequal counts, block_2_load_odl_data.py:31-38; matrix lists may
hold any matrices): each distinct operator is one device batch (groups.RankGroups).
One process per GPU: when
``torch.distributed`` is initialised with world size > 1 the graph nodes are
sharded (plan.py) and every rank returns the same ``(x_list, history)``.
"""
from __future__ import annotations

import math
import os
from datetime import datetime

import numpy as np
import torch
import torch.distributed as dist

from .exchange import split_stats
from .geometry import RayTransform
from .groups import RankGroups
from .matrix import MatrixOperator, as_operators

HISTORY_KEYS = (
    "primal", "dual", "pri_per_node", "dual_per_node", "obj_per_node", "obj_total",
    "mse_sino_per_node", "mse_sino_total", "img_mse_per_node", "img_mse_total",
    "g_norm_history", "eps_used_history", "eps_target_history",
)

EXTRA_KEYS = ("sb_res_history", "inner_updates_history")

DEFAULT_MU_FACTOR = 10.0  # split-Bregman penalty mu = 10 * lam_tv
EPS_CAP, CALIB_ALPHA, MAX_TIGHTEN = 1e-2, 1.0, 2  # block_6_admm_loop_ver2.py:106-113
PIPELINE_BLOCK = 64  # iterations of statistics held on the device in the pipelined mode


def eps_target(k: int) -> float:
    """block_6_admm_loop_ver2.py:101-103."""
    return 2.0 / ((k + 1) ** 1.005)


def _check_operators(A_list, N):
    """Every entry an admm_hip operator on an N x N image.  Nodes may have different
    operators (unequal angle counts, different matrices): RankGroups batches equal ones."""
    for A in A_list:
        if not isinstance(A, (RayTransform, MatrixOperator)):
            raise TypeError(
                "A_dense_list entries must be admm_hip operators (RayTransform, MatrixOperator) "
                f"or matrices; got {type(A).__name__}")
        if A._adjoint:
            raise ValueError("A_dense_list entry is an adjoint view")
        if A.geom.N != N:
            raise ValueError(f"N={N} does not match an operator's N={A.geom.N}")


def _dist_info(group):
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def run_admm(A_dense_list, sinograms, G, Wi_list, Qij_diag_fn, N, lam_tv=0.01, rho=1.0,
             max_iters=10, eps_pri=1e-1, eps_dual=1e-1, verbose=True, snapshot_dir=None,
             snapshot_every=None, snapshot_div=10, phantom_true=None, mu=None, tv_iters=10,
             cg_iters=5, tv_kind="iso", group=None, return_tensors=False, timing=None,
             write_params=True, fusion="midpoint", inner_tol=None, max_inner_updates=10,
             inner_chunks=None, chunk_snapshot_dir=None, chunk_save_every=1, inspect=None,
             pipeline=None, streams=1, edge_state=None):
    """``edge_state``: "stored" / "derived" z (None: the run's rule, plan.z_is_stored --
    stored wherever it fits; ADMM_EDGE_STATE in the environment forces it too).
``inner_chunks``: split each x-update into warm-started solves of these round counts
    (block_6_admm_loop.py:14-69 chunked SCS); ``chunk_snapshot_dir`` then receives that
    file's per-chunk snapshots (``_chunk_snapshot``) every ``chunk_save_every`` chunks.
    ``inspect(rg)``: called with the rank's device state (groups.RankGroups) after the loop
    (tests check the edge invariants on the device arrays).  ``pipeline``: read the
    statistics back once after the loop instead of every iteration (default: whenever the
    stop test cannot fire and no per-iteration host output is requested; False forces the
    per-iteration read-back).  ``streams``: concurrent node batches per rank (groups.RankGroups;
    bitwise the same run).  In the pipelined mode the device keeps the statistics of at most
    ``PIPELINE_BLOCK`` iterations (V_total x 8 + E x 3 float64 each) and flushes them to the host
    every ``PIPELINE_BLOCK`` iterations, so the verbose progress lines of those iterations are
    printed at each flush (and at the end), not as each iteration finishes."""
    if inner_tol not in (None, "reference"):
        raise ValueError("inner_tol must be None (fixed counts) or 'reference'")
    if inner_chunks is not None:
        inner_chunks = [int(r) for r in inner_chunks]
        if not inner_chunks or min(inner_chunks) < 1:
            raise ValueError("inner_chunks must be a non-empty list of positive round counts")
        if inner_tol is not None:
            raise ValueError("inner_chunks and inner_tol are exclusive")
        tv_iters = inner_chunks[0]
    V_total = len(A_dense_list)
    # matrices (the reference's dense A_dense_list; dense numpy / torch, scipy.sparse)
    # become explicit-matrix operators (matrix.py); operators pass through
    A_dense_list = as_operators(A_dense_list, N=N)
    _check_operators(A_dense_list, N)
    if sorted(G.nodes()) != list(range(V_total)):
        raise ValueError("graph nodes must be 0..num_nodes-1")
    mu = DEFAULT_MU_FACTOR * lam_tv if mu is None else float(mu)
    if not mu > 0:
        raise ValueError("mu must be > 0 (set lam_tv > 0 or pass mu explicitly)")
    world, rank = _dist_info(group)
    torch.cuda.set_device(A_dense_list[0].device)
    if snapshot_dir is not None:
        os.makedirs(snapshot_dir, exist_ok=True)
    if snapshot_every is None:
        snapshot_every = max(1, max_iters // snapshot_div)  # _ver2:31-32
    rg = RankGroups(A_dense_list, G, V_total, world, rank, sinograms, Qij_diag_fn, rho, lam_tv, mu,
                    tv_iters, cg_iters, tv_kind, phantom_true, fusion=fusion, Wi_list=Wi_list,
                    keep_x=inner_tol is None, group=group, streams=streams,  # this loop never writes x itself
                    derive_z=None if edge_state is None else {"stored": False, "derived": True}[edge_state])
    # (masked re-solves of the tolerance mode restore x rows, so that mode re-projects x)
    plan = rg.plan
    if world > 1:
        dist.barrier(group=group)
    hist = {k: [] for k in HISTORY_KEYS + EXTRA_KEYS}
    edges = plan.edges
    have_ph = phantom_true is not None
    if verbose and rank == 0:
        print(f"Max ADMM Iteration in Block-6 B4 Loop = {max_iters}")
    torch.cuda.synchronize()
    t_loop = None
    if timing is not None:
        import time
        t_loop = time.perf_counter()
    iters_done = 0
    # Pipelined statistics: when the stop test cannot fire (eps_pri <= 0 or eps_dual <= 0:
    # primal / dual are norms) and nothing else needs host values per iteration, each
    # iteration's statistics table is assembled on the device (RCCL all-reduce at N > 1) into
    # a row of a device history and read back once after the loop -- no host synchronisation
    # per iteration, so the next iteration's launches queue behind the current one.  The
    # histories are computed from the same values by the same host code (bitwise equal).
    pipelined = ((eps_pri <= 0 or eps_dual <= 0) and inner_tol is None and snapshot_dir is None
                 and chunk_snapshot_dir is None and pipeline is not False)
    dev_hist = None
    flushed = 0  # iterations of the pipelined statistics already recorded on the host
    for k in range(max_iters):
        et = eps_target(k)
        if inner_chunks is None:
            rg.node_update()
        else:
            for cid, rounds in enumerate(inner_chunks):
                rg.node_update(rounds=rounds)
                if chunk_snapshot_dir is not None and cid % int(chunk_save_every) == 0:
                    _chunk_snapshot(chunk_snapshot_dir, k, cid, rg, N)
        eps_used = np.full(plan.V, np.nan)
        n_upd = np.ones(plan.V)
        if inner_tol == "reference":
            for nb in rg.batches:
                rows = [plan.local_nodes.index(g) for g in nb.plan.local_nodes]
                eps_used[rows], n_upd[rows] = _solve_to_reference_tolerance(nb, et, max_inner_updates)
        rg.exchange_consensus()  # (rank-internal edges under the halo exchange)
        iters_done = k + 1
        if pipelined:
            flat = rg.stats_device()
            if dev_hist is None:
                dev_hist = torch.empty((min(max_iters, PIPELINE_BLOCK), flat.numel()), dtype=torch.float64,
                                       device=flat.device)
            dev_hist[k - flushed].copy_(flat)
            if k + 1 - flushed == dev_hist.shape[0]:  # block full: flush to the host
                flushed = _flush_pipelined(hist, dev_hist, flushed, k + 1, rg, V_total, edges, rho, lam_tv,
                                           have_ph, verbose and rank == 0)
            continue
        ns, es = rg.stats(np.stack([eps_used, n_upd], axis=1))
        pn, dn = _record(hist, ns.numpy(), es.numpy(), edges, V_total, rho, lam_tv, et, have_ph)
        if snapshot_dir is not None and ((k + 1) % snapshot_every == 0):
            _snapshot(snapshot_dir, k, rg, N)
        if verbose and rank == 0 and k % 10 == 0:
            print(f"iter {k}, primal {pn:.3e}, dual {dn:.3e}")
        if pn < eps_pri and dn < eps_dual:
            if verbose and rank == 0:
                print(f"stopped at iter {k}, primal {pn:.3e}, dual {dn:.3e}")
            break
    if pipelined and dev_hist is not None and iters_done > flushed:
        flushed = _flush_pipelined(hist, dev_hist, flushed, iters_done, rg, V_total, edges, rho, lam_tv, have_ph,
                                   verbose and rank == 0)
    torch.cuda.synchronize()
    if timing is not None:
        import time
        timing["loop_s"] = time.perf_counter() - t_loop
        timing["iters"] = iters_done
        timing["V_total"] = V_total
    if write_params and rank == 0:
        _write_params(snapshot_dir, rho, lam_tv, V_total, mu, tv_iters, cg_iters)
    if inspect is not None:
        inspect(rg)
    X = rg.images()
    if return_tensors:
        return [X[i] for i in range(V_total)], hist
    Xh = X.to("cpu").numpy()
    return [Xh[i].copy() for i in range(V_total)], hist


def _flush_pipelined(hist, dev_hist, k0, k1, rg, V_total, edges, rho, lam_tv, have_ph, verbose):
    """Record iterations k0 .. k1-1 of the pipelined statistics (rows 0 .. k1-k0-1 of
    ``dev_hist``) on the host; returns k1."""
    host = dev_hist[: k1 - k0].to("cpu")
    nsw = rg.batches[0].node_stats.shape[1]
    extra = np.stack([np.full(V_total, np.nan), np.ones(V_total)], axis=1)
    for k in range(k0, k1):
        ns, es = split_stats(host[k - k0], V_total, nsw, len(edges), rg.batches[0].edge_stats.shape[1])
        pn, dn = _record(hist, np.concatenate([ns.numpy(), extra], axis=1), es.numpy(), edges, V_total,
                         rho, lam_tv, eps_target(k), have_ph)
        if verbose and k % 10 == 0:
            print(f"iter {k}, primal {pn:.3e}, dual {dn:.3e}")
    return k1


def _record(hist, ns, es, edges, V_total, rho, lam_tv, et, have_ph):
    """Append one iteration's histories from the global statistics tables (nodes x 8, edges x 3);
    returns (primal, dual)."""
    # --- node diagnostics (_ver2:145-206) ---
    mse = ns[:, 0].copy()
    g_norm = np.sqrt(ns[:, 1])
    obj = 0.5 * ns[:, 0] + lam_tv * ns[:, 2] + ns[:, 3]
    hist["g_norm_history"].append(g_norm)
    hist["eps_used_history"].append(ns[:, 6].copy())
    hist["eps_target_history"].append(np.full(V_total, et))
    hist["sb_res_history"].append(np.sqrt(ns[:, 5]))
    hist["inner_updates_history"].append(ns[:, 7].astype(np.int64))
    hist["mse_sino_per_node"].append(mse)
    hist["mse_sino_total"].append(float(np.sum(mse)))
    img = ns[:, 4].copy() if have_ph else np.full(V_total, np.nan)
    hist["img_mse_per_node"].append(img)
    hist["img_mse_total"].append(float(np.sum(img)))
    # --- residuals in G.edges() order (_ver2:232-258) ---
    r2 = 0.0
    s2 = 0.0
    pri = np.zeros(V_total)
    dua = np.zeros(V_total)
    for ge, (a, b) in enumerate(edges):
        ra2, rb2, dz2 = float(es[ge, 0]), float(es[ge, 1]), float(es[ge, 2])
        r2 += ra2 + rb2
        pri[a] += ra2
        pri[b] += rb2
        s2 += rho * rho * dz2
        dua[a] += rho * rho * dz2
        dua[b] += rho * rho * dz2
    pn, dn = math.sqrt(r2), math.sqrt(s2)
    hist["primal"].append(pn)
    hist["dual"].append(dn)
    hist["obj_per_node"].append(obj)
    hist["obj_total"].append(float(np.sum(obj)))
    hist["pri_per_node"].append(np.sqrt(pri))
    hist["dual_per_node"].append(np.sqrt(dua))
    return pn, dn


def _solve_to_reference_tolerance(nb, et, max_inner_updates):
    """block_6_admm_loop_ver2.py:105-176 for every local node (after its first x-update):
    solve to eps_try, accept if ||g|| <= eps_target, else tighten eps_try /= 5 (<= 2 times)."""
    V = nb.V
    eps_try = np.full(V, min(EPS_CAP, CALIB_ALPHA * et))
    tries = np.zeros(V, dtype=np.int64)
    n_upd = np.ones(V)
    active = np.ones(V, dtype=bool)
    st = nb.node_stats.to("cpu").numpy()
    while True:
        g, sb = np.sqrt(st[:, 1]), np.sqrt(st[:, 5])
        need = active & (sb > eps_try) & (n_upd < (tries + 1) * max_inner_updates)
        if need.any():  # keep solving the nodes not yet at their eps_try
            nb.node_update_masked(need)
            n_upd += need
            st = nb.node_stats.to("cpu").numpy()
            continue
        done = active & ((g <= et) | (tries >= MAX_TIGHTEN))  # accepted or forced (:155-172)
        active &= ~done
        if not active.any():
            return eps_try, n_upd
        tries[active] += 1
        eps_try[active] /= 5.0  # :174-176


def _chunk_snapshot(out_dir, k, cid, rg, N):
    """block_6_admm_loop.py:55-66: {out_dir}/node_{i}/node_{i}_outer_{k}_chunk_{c}.npy holding
    x.reshape(N, N, order="F") (the skeleton's Fortran-order image), + .png."""
    plt = _pyplot()
    for g, xr in rg.local_images():
        d = os.path.join(out_dir, f"node_{g}")
        os.makedirs(d, exist_ok=True)
        tag = f"node_{g}_outer_{k}"
        img = xr.to("cpu").numpy().reshape(N, N, order="F")
        np.save(os.path.join(d, f"{tag}_chunk_{cid}.npy"), img)
        if plt is not None:
            plt.figure(figsize=(5, 5))
            plt.imshow(img, cmap="gray")
            plt.title(f"{tag} after chunk {cid}")
            plt.axis("off")
            plt.tight_layout()
            plt.savefig(os.path.join(d, f"{tag}_chunk_{cid}.png"), dpi=220)
            plt.close()


def _pyplot():
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        return plt
    except Exception:  # pragma: no cover
        return None


def _snapshot(snapshot_dir, k, rg, N):
    """_ver2:269-281: iter_XXXX_node_i.npy (C-order reshape) + .png."""
    it_tag = f"iter_{k + 1:04d}"
    plt = _pyplot()
    for g, xr in rg.local_images():
        img = xr.to("cpu").numpy().reshape(N, N)
        np.save(os.path.join(snapshot_dir, f"{it_tag}_node_{g}.npy"), img)
        if plt is not None:
            plt.figure(figsize=(5, 5))
            plt.imshow(img, cmap="gray")
            plt.title(f"{it_tag}  node {g}")
            plt.axis("off")
            plt.tight_layout()
            plt.savefig(os.path.join(snapshot_dir, f"{it_tag}_node_{g}.png"), dpi=220)
            plt.close()


def _write_params(snapshot_dir, rho, lam_tv, V, mu, tv_iters, cg_iters):
    """_ver2:291-306 admm_internal_params.txt."""
    try:
        log_dir = snapshot_dir if snapshot_dir is not None else os.getcwd()
        os.makedirs(log_dir, exist_ok=True)
        with open(os.path.join(log_dir, "admm_internal_params.txt"), "w") as f:
            f.write("===== ADMM Internal Parameters =====\n")
            f.write(f"rho = {rho}\n")
            f.write(f"lambda_tv = {lam_tv}\n")
            f.write(f"Number of nodes = {V}\n")
            f.write("Calib alpha = 1.0\n")
            f.write("Eps cap = 0.01\n")
            f.write(f"Split-Bregman mu = {mu}\n")
            f.write(f"Inner iterations (tv x cg) = {tv_iters} x {cg_iters}\n")
            f.write(f"Date-Time: {datetime.now().strftime('%Y-%m-%d %H:%M:%S')}\n")
    except Exception as e:  # pragma: no cover
        print(f"[WARN] Could not save internal params: {e}")
