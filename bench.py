"""Benchmark: decentralized-ADMM node-updates/s on MI355X (BASELINE.json metric).

Headline workload (``--workload auto``):

* one GPU: BASELINE.json configs[2] itself -- C3: 512^2 modified Shepp-Logan, a 16-node
  ring, 96 angles per node (1536 = 3N in total), float32 projector samples / float64
  solver state, lambda_TV = 0.02, rho = 2, split-Bregman 10 rounds x 5 CG steps per
  x-update;
* N > 1 GPUs (weak scaling, one process per GPU): the same per-node problem with 8 graph
  nodes per GPU on a ring of 8N (N = 2 is C3 sharded over 2 GPUs exactly, as configs[2]
  specifies).  The line also carries ``weak8`` at one GPU (8 nodes, the per-GPU share of
  the N > 1 runs) and the strong-scaling legs ``strong`` (C3 and C4 -- 1024^2, 32-node
  Erdos-Renyi graph -- sharded over the same N ranks; at one GPU only C4, C3 being the
  headline).

A "step" is one outer ADMM iteration: the x-update of every node, the halo exchange
(RCCL), the z/y edge updates and the residual/statistics readback the reference's stop
test needs (asynchronous, into pinned host memory: run_admm's pipelined mode, DESIGN.md
section 9).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--strong C3,C4|none] [--proxy fast|all|none]
    torchrun --nproc-per-node N bench.py --gpus N ...
    python bench.py --config C2|C3|C4|C5|C5s [--as-rank R/W]

``python bench.py --gpus N`` with N > 1 and no WORLD_SIZE in the environment launches
the N ranks itself (one child process per GPU, RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR=127.0.0.1 / MASTER_PORT set; the parent makes no GPU call), relays rank 0's
line and exits non-zero if any rank fails.  Under a launcher, --gpus must equal WORLD_SIZE.

Per-rank proxies (``proxy_8gpu``, one GPU only).  The multi-GPU runs shard graph nodes,
and every rank's x-updates are independent within an iteration
(block_6_admm_loop_ver2.py:81-97), so rank R of a W-rank run does exactly its own share:
its contiguous node block (one device batch at its own node-interleave width, e.g. 4
nodes at VB = 4 for C4 on 8 GPUs), every halo row and every stored edge of
plan.make_plan(G, V, W, R).  A proxy binds that share on this one GPU and times
x-update + consensus + statistics with the halo rows held fixed; the exchange is
priced from its bytes over xGMI (7 links x 153 GB/s per MI355X, task spec): ``direct``
spreads the received bytes over min(peers, 7) links, ``one_link`` puts them on one.
predicted_speedup = T_1 / (T_rank + t_exchange), T_1 = the config on one GPU (measured
in the same run); ``per_node_cost_ratio`` = (T_rank / V_rank) / (T_1 / V).  ``--as-rank
R/W`` with ``--config`` prints one such share as its own line.

Roofline (``roofline``): the dominant kernel -- of the two projectors, each launched once
per CG step, the one with the longer in-solve launch (at C3 the back projector
k_back_mirror in H mode, ahead of the forward taps k_fwdg); both are reported as
``roofline_back`` and ``roofline_fwd``.  A kernel's average launch duration is measured live
with HIP events on the stream it runs on, around each of its in-solve launches; its HBM bytes
per launch come from the committed rocprofv3 PMC passes (2 x FETCH_SIZE + WRITE_SIZE,
MI355X_MICROARCH.md) of the in-solve launches of the same workload (TRAFFIC_FILES), so
``frac`` = PMC bytes / live duration / 8 TB/s.  ``compulsory_bytes`` is what one launch must
move at least; ``lds`` puts the tap reads (LDS-served) against the aggregate ds_read_b128
rate; ``sample_touch`` is SURVEY.md 8d's per-tap accounting, which counts LDS-served taps
and so exceeds any memory peak -- a reuse factor, not a rate.  ``step_hbm`` is the whole
step's PMC traffic over the measured step time.

CPU baseline (``cpu_baseline``): the float64 NumPy/SciPy oracle (oracle/, the port of
the reference algorithm -- the reference's CVXPY/ODL path cannot run here) doing the
SAME first x-update of node 0 (the GPU's own float32 sinogram, precisions and zero
start) in one process per host core; ``rel_fro`` = GPU node-0 image vs that oracle image;
``eq1_gap`` = that image's certified distance from eq.(1)'s exact minimiser (oracle/eq1.py).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-inverse-problem-admm_amd"))
sys.path.insert(0, ROOT)

N_IMG = 512
NODES_PER_GPU = 8  # weak-scaling share at N > 1 GPUs
ANGLES_PER_NODE = 96
LAM, RHO = 0.02, 2.0
TV_ITERS, CG_ITERS = 10, 5
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
LDS_PEAK_GBS = 150000.0  # aggregate ds_read_b128 rate, every CU streaming (MI355X_MICROARCH.md, LDS)
CPU_BASELINE_SECONDS = 8.0  # per-process compute budget of the bounded CPU sample
XGMI_LINK_GBS, XGMI_LINKS = 153.0, 7  # per direction per link, links per MI355X (task spec)
RCCL_CALL_US = 50.0  # assumed fixed cost per RCCL call per iteration (launch + handshake), conservative model


# BASELINE.json configs[1..4]: image side, total graph nodes, graph, dtype, TV
CONFIGS = {
    "C2": dict(N=256, nodes=8, graph="ring", dtype="float32", tv="iso"),
    "C3": dict(N=512, nodes=16, graph="ring", dtype="float32", tv="iso"),
    "C4": dict(N=1024, nodes=32, graph="er", dtype="float32", tv="iso"),
    "C5": dict(N=2048, nodes=64, graph="complete", dtype="float64", tv="aniso"),
    # C5's per-GPU share (8 of its 64 nodes at 8 GPUs) on one GPU: a 1-GPU rehearsal of the
    # 2048^2 float64 anisotropic x-update (complete graph of the 8 local nodes)
    "C5s": dict(N=2048, nodes=8, graph="complete", dtype="float64", tv="aniso", angles_per_node=96),
}
BASELINE_INDEX = {"C2": 1, "C3": 2, "C4": 3, "C5": 4}


def workload_cfg(name, world=1):
    """A BASELINE config, or ``weak8``: 8 nodes per GPU on a ring of 8 x world (512^2, 96
    angles per node; world = 2 is C3)."""
    if name == "weak8":
        return dict(N=N_IMG, nodes=NODES_PER_GPU * world, graph="ring", dtype="float32", tv="iso",
                    angles_per_node=ANGLES_PER_NODE)
    return CONFIGS[name]


def make_graph(kind, V):
    import math
    import networkx as nx
    if kind == "ring":
        return nx.cycle_graph(V)
    if kind == "complete":
        return nx.complete_graph(V)
    # Erdos-Renyi p = 2 ln V / V, seed 0, resampled (seed + 1) until connected
    p = 2.0 * math.log(V) / V
    seed = 0
    while True:
        G = nx.erdos_renyi_graph(V, p, seed=seed)
        if nx.is_connected(G):
            return G
        seed += 1


def sample_touch_bytes(N, a, tv, cg, sample_bytes=4):
    """SURVEY.md 8d sample-touch bytes: (B_A, B_At, B_node) per node (4-byte samples, 8 in C5)."""
    m = a * N
    n = N * N
    sb = sample_bytes
    B_A = sb * m * (2 * N + 1)
    B_At = sb * n * (2 * a + 1)
    B_cg = B_A + B_At + 6 * sb * n + 14 * sb * n
    return B_A, B_At, tv * (cg * B_cg + 27 * sb * n) + B_At + sb * n * (3 * 2 + 2)


# ---------------------------------------------------------------------------
# CPU baseline: the oracle's x-update, one spawned process per host core
# ---------------------------------------------------------------------------
def _cpu_worker(wid, N, a, b, q, budget, barrier, out):
    """One process: build the Joseph CSR matrix, wait for the others, run x-updates of
    node 0's first ADMM iteration (zero start, v = 0) until ``budget`` seconds pass."""
    import numpy as np
    from oracle import node_solver as ons
    from oracle.geometry import Geometry, joseph_matrix
    A = joseph_matrix(Geometry(N, a))
    AT = A.T.tocsr()
    b = np.asarray(b, dtype=np.float64)
    q = np.asarray(q, dtype=np.float64)
    Atb = AT @ b
    n = N * N
    v = np.zeros(n)
    prm = ons.NodeParams(rho=RHO, lam=LAM, mu=10 * LAM, tv_iters=TV_ITERS, cg_iters=CG_ITERS)
    barrier.wait()
    t0 = time.perf_counter()
    done, x, st0 = 0, None, None
    while True:
        st = ons.NodeState.zeros(n)
        ons.node_update(A, Atb, b, 2 * q, 2 * q * v, [(q, v), (q, v)], st, N, prm, AT=AT)
        done += 1
        el = time.perf_counter() - t0
        if x is None:
            x, st0 = st.x, st
        if el >= budget:
            break
    cert = None
    if wid == 0:
        # eq.(1)'s optimality certificate for the oracle image (after the timed region): with
        # the split-Bregman dual p = mu e / lam and m = rho min(D) <= lambda_min(H),
        # ||x - x*|| <= (||r|| + sqrt(||r||^2 + 2 m eps)) / m  (oracle/eq1.py)
        from oracle import eq1
        D = 2 * q
        delta, gap, rn, eps = eq1.certificate(A, b, D, 2 * q * v, st0.x, prm.mu * st0.ex / prm.lam,
                                              prm.mu * st0.ey / prm.lam, N, prm.rho, prm.lam, "iso")
        f = ons.objective(A, b, st0.x, N, prm.rho, prm.lam, [(q, v), (q, v)], "iso")  # eq.(1) at x
        cert = dict(dist_bound=delta, rel_dist_bound=delta / float(np.linalg.norm(st0.x)), obj_gap_bound=gap,
                    objective=f, rel_obj_gap_bound=gap / f, stationarity=rn, eps=eps, m=float(prm.rho * D.min()))
    out.put((wid, done, el, x if wid == 0 else None, cert))


def cpu_baseline(N, a, b, q, x_gpu, procs=None, budget=CPU_BASELINE_SECONDS):
    """Oracle x-updates of node 0 on ``procs`` host processes (one per core, 1 thread each).

    value = updates completed by all processes / the slowest process's compute time
    (matrix builds excluded); rel_fro = ||x_gpu - x_oracle|| / ||x_oracle||."""
    import multiprocessing as mp
    import numpy as np
    if procs is None:
        cap = int(os.environ.get("ADMM_CPU_BASELINE_PROCS", os.environ.get("OMP_NUM_THREADS", "0")) or 0)
        procs = os.cpu_count() or 1
        if cap > 0:
            procs = min(procs, cap)
    ctx = mp.get_context("spawn")  # fresh interpreters: nothing of this process's GPU state
    saved = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")}
    for k in saved:
        os.environ[k] = "1"
    try:
        barrier = ctx.Barrier(procs)
        out = ctx.Queue()
        ps = [ctx.Process(target=_cpu_worker, args=(w, N, a, b, q, budget, barrier, out)) for w in range(procs)]
        t0 = time.perf_counter()
        for p in ps:
            p.start()
        res = [out.get() for _ in ps]
        for p in ps:
            p.join()
        wall = time.perf_counter() - t0
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    done = sum(r[1] for r in res)
    el = max(r[2] for r in res)
    x_cpu = next(r[3] for r in res if r[0] == 0)
    cert = next(r[4] for r in res if r[0] == 0)
    rel = float(np.linalg.norm(x_gpu - x_cpu) / np.linalg.norm(x_cpu))
    return {"value": done / el, "unit": "node-updates/s", "cores": procs, "kind": "port",
            "rel_fro": rel,
            "eq1_gap": dict(cert, note="certified distance of the oracle's node-0 image (the iteration the "
                                       "GPU matches to rel_fro) from eq.(1)'s exact minimiser "
                                       "(block_5_node_problem.py:21-29): split-Bregman dual p = mu e / lam, "
                                       "strong convexity m = rho min(D) (a lower bound on lambda_min(H)); "
                                       "obj_gap_bound = ||r||^2 / 2m + eps >= f(x) - f(x*), objective = f(x) (eq.(1)), "
                                       "rel_obj_gap_bound = obj_gap_bound / f(x); the reference's "
                                       "SCS solve is inexact too (eps = min(1e-2, eps_target))"),
            "sample": f"{done} x-updates of node 0's first ADMM iteration ({N}^2, {a} angles, 2 ring "
                      f"neighbours, 10x5 inner, zero start) on the GPU run's own float32 sinogram "
                      f"and precisions; float64 SciPy CSR Joseph oracle, {procs} processes x 1 "
                      f"thread, {el:.1f} s of compute (CSR builds excluded; {wall:.1f} s wall); "
                      f"rel_fro = GPU node-0 image vs the oracle image"}


# ---------------------------------------------------------------------------
# PMC traffic (committed rocprofv3 passes)
# ---------------------------------------------------------------------------
# HBM bytes per forward-projector launch and per step from the committed rocprofv3 PMC
# summaries (scripts/pmc.sh + scripts/traffic_summary.py over the launches between the
# bench's markers, i.e. the timed steps; 2 x FETCH_SIZE + WRITE_SIZE per the
# MI355X_MICROARCH.md gfx950 correction), one per headline workload: the per-launch
# figure depends on the node chunks one launch projects.  PMC counters cannot be read
# inside this run.
TRAFFIC_FILES = {"C3": "profiles/r6_traffic.json", "weak8": "profiles/r6_traffic_weak8.json"}


def fwd_kernel_name(tr, tname, vb, mirror):
    """The batch's forward projector instantiation as rocprofv3 names it: k_fwdg<T, VB, MIRROR,
    VBR, CPB> (mirror mode projects virtual width 2 x VBR; CPB = 2 virtual chunks per block where
    the halved block table fills the chip); with a traffic file, the one that ran."""
    head = f"admm::k_fwdg<{tname}, {min(2 * vb, 32 // (8 if tname == 'double' else 4)) if mirror else vb}, " \
           f"{'true' if mirror else 'false'}, {vb}"
    names = [f"{head}, 2>", f"{head}, 1>", f"{head}>"]
    kern = (tr or {}).get("kernels", {})
    return next((n for n in names if n in kern), names[1])


def fwd_kernel_traffic(tr, tname, vb, mirror):
    """PMC bytes per launch of the batch's forward projector (fwd_kernel_name)."""
    if not tr:
        return None
    return tr["kernels"].get(fwd_kernel_name(tr, tname, vb, mirror), {}).get("hbm_bytes_per_launch")


KERNEL_SOURCES = ("distributed-inverse-problem-admm_amd/csrc/kernels.hpp",
                  "distributed-inverse-problem-admm_amd/csrc/admm_tomo.hip")


def kernel_source_sha16():
    """sha256 (first 16 hex digits) of the kernel sources the library is built from; a PMC
    traffic file records the hash of the sources it measured (scripts/traffic_summary.py)."""
    import hashlib
    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        with open(os.path.join(ROOT, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


TRAFFIC_STALE = {}  # workload -> why its traffic file was not used


def pmc_traffic(workload):
    """The committed PMC traffic of ``workload`` -- only if it was measured on kernels built
    from the current sources (same kernel_source_sha16); otherwise (None, file) and the reason
    in TRAFFIC_STALE: the line then carries traffic null rather than bytes of older kernels."""
    f = TRAFFIC_FILES.get(workload)
    if f is None:
        return None, None
    try:
        with open(os.path.join(ROOT, f)) as fh:
            tr = json.load(fh)
    except (OSError, ValueError):
        TRAFFIC_STALE[workload] = f"{f}: missing or unreadable"
        return None, f
    want, have = kernel_source_sha16(), tr.get("kernel_source_sha16")
    if have != want:
        TRAFFIC_STALE[workload] = (f"{f} measured kernels of source hash {have}, the library is built from "
                                   f"{want}: traffic not reused")
        return None, f
    return tr, f


STREAMS = 1  # concurrent batch streams per rank (--streams; RankGroups)
EDGE_STATE = None  # --edge-state stored|derived forces z's form (default: the run's rule, plan.z_is_stored)


def setup_run(name, world, rank, local_rank, exchange=True):
    """Operators, sinograms, precisions and the bound node batches of rank ``rank`` of a
    ``world``-rank run of workload ``name``.  ``exchange=False``: no inter-rank exchange (a
    per-rank proxy on one GPU; halo rows held fixed)."""
    from admm_hip.data import make_precisions, make_sinograms, shepp_logan
    from admm_hip.groups import RankGroups
    from admm_hip.plan import make_plan
    from admm_hip.solver import make_operators
    cfg = workload_cfg(name, world)
    n_img, V_total, dtype, tv_kind = cfg["N"], cfg["nodes"], cfg["dtype"], cfg["tv"]
    G = make_graph(cfg["graph"], V_total)
    angles_total = max(180, 3 * n_img)  # block_2_load_odl_data.py:31-38
    if "angles_per_node" in cfg:  # a share of a larger config keeps its per-node angle count
        angles_total = cfg["angles_per_node"] * V_total
    ops = make_operators(n_img, V_total, angles_total=angles_total, dtype=dtype, device=local_rank)
    geom = ops[0].geom
    local = make_plan(G, V_total, world, rank).local_nodes
    ph = shepp_logan(n_img)
    sinos = dict(zip(local, make_sinograms([ops[g] for g in local], ph, 0.005, seed=1000 + local[0])))
    Wi, Q = make_precisions(ops)  # one W kernel launch: every node shares the geometry
    rg = RankGroups(ops, G, V_total, world, rank, sinos, Q, RHO, LAM, 10 * LAM, TV_ITERS, CG_ITERS, tv_kind, ph,
                    keep_x=True, halo=exchange, streams=STREAMS,
                    derive_z=None if EDGE_STATE is None else EDGE_STATE == "derived")
    return dict(name=name, n_img=n_img, V_total=V_total, dtype=dtype, tv_kind=tv_kind, geom=geom, plan=rg.plan,
                rg=rg, nb=rg.batches[0], Wi=Wi, graph=cfg["graph"])


def timed_steps(r, steps, warmup, world, prime=None, markers=False):
    """Warmup + K timed outer iterations (barrier + synchronize on both sides, max over
    ranks; ``world`` = this job's process count).  ``prime(nb)`` runs right after the first
    x-update (before its exchange).  ``markers`` with ADMM_BENCH_MARKERS=1: one marker kernel
    on each side of the timed steps (scripts/pmc.sh's PMC window)."""
    import torch
    import torch.distributed as dist
    rg = r["rg"]
    host = None

    def step(first=False):
        nonlocal host
        rg.node_update()
        if first and prime is not None:
            prime(rg.batches[0])
        rg.exchange_consensus()  # (rank-internal edges under the halo exchange)
        # the statistics the stop test reads (global table, RCCL all-reduce at N > 1), read
        # back every step into pinned host memory without a per-step host synchronisation --
        # run_admm's pipelined mode (the stop test cannot fire at eps = 0)
        flat = rg.stats_device() if world > 1 or rg.halo is not None else _stats_local(rg)
        if host is None:
            host = torch.empty(flat.shape, dtype=flat.dtype, pin_memory=True)
        host.copy_(flat, non_blocking=True)

    step(first=True)  # the first (full-projection) x-update; later ones replay the reuse graph
    for _ in range(max(0, warmup - 1)):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    marks = markers and os.environ.get("ADMM_BENCH_MARKERS") == "1"
    if marks:
        rg.batches[0].marker()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if marks:
        rg.batches[0].marker()
        torch.cuda.synchronize()
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el


def _stats_local(rg):
    """A proxy rank's statistics table (its own rows of the global one; the W-rank run adds
    one all-reduce of (V x 8 + E x 3) doubles, which the proxy prices with the exchange)."""
    from admm_hip.exchange import assemble_stats_device
    parts = [(nb.plan, nb.node_stats, nb.edge_stats[: len(nb.plan.stored_edges)]) for nb in rg.batches]
    return assemble_stats_device(rg.plan.V_total, len(rg.plan.edges), 1, parts)


# ---------------------------------------------------------------------------
# per-rank proxies of the multi-GPU runs
# ---------------------------------------------------------------------------
def exchange_model(plan, n_img):
    """Bytes one rank receives per iteration in ``plan``'s exchange and their xGMI time
    (float64 images; the all-gather moves every rank's padded block, p2p only halo rows)."""
    npx = n_img * n_img
    if plan.world == 1:
        return {"mode": "none", "bytes_received": 0, "peers": 0, "ms_direct": 0.0, "ms_one_link": 0.0}
    stats_bytes = 8 * (plan.V_total * 8 + len(plan.edges) * 3)  # statistics all-reduce
    if plan.use_allgather():
        vmax = max(hi - lo for lo, hi in plan.ranges)
        recv = (plan.world - 1) * vmax * npx * 8
        peers = plan.world - 1
        mode = "allgather"
    else:
        recv = sum(len(v) for v in plan.recv.values()) * npx * 8
        peers = sum(1 for v in plan.recv.values() if v)
        mode = "p2p"
    links = max(1, min(peers, XGMI_LINKS))
    calls = 2  # the halo exchange (one all-gather, or one grouped p2p batch) + the statistics all-reduce
    lat = calls * RCCL_CALL_US * 1e-3
    return {"mode": mode, "bytes_received": recv, "peers": peers, "stats_bytes": stats_bytes,
            "rccl_calls": calls,
            "ms_direct": 1e3 * (recv + stats_bytes) / (links * XGMI_LINK_GBS * 1e9),
            "ms_one_link": 1e3 * (recv + stats_bytes) / (XGMI_LINK_GBS * 1e9),
            # conservative: every received byte over ONE link, plus a fixed cost per RCCL call
            "ms_conservative": 1e3 * (recv + stats_bytes) / (XGMI_LINK_GBS * 1e9) + lat}


def busiest_rank(name, world):
    """The rank of a ``world``-rank run with the most local nodes, then stored edges, then
    halo rows (the slowest share, which sets the max-over-ranks step time)."""
    from admm_hip.plan import make_plan
    cfg = workload_cfg(name, world)
    G = make_graph(cfg["graph"], cfg["nodes"])
    best, key = 0, None
    for r in range(world):
        p = make_plan(G, cfg["nodes"], world, r)
        k = (p.V, len(p.stored_edges), len(p.halo_nodes))
        if key is None or k > key:
            best, key = r, k
    return best


def time_share(name, world, rank, steps, warmup):
    """Rank ``rank``'s share of a ``world``-rank run of ``name``, timed on this GPU; also the
    edge updates alone (``consensus_ms``: consensus + statistics, event-timed)."""
    import torch
    r = setup_run(name, world, rank, 0, exchange=False)
    el = timed_steps(r, steps, max(warmup, 3), 1)  # (>= 2 replays of the reuse graph before timing)
    plan, nb = r["plan"], r["nb"]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    reps = 5
    ev[0].record()
    for _ in range(reps):
        r["rg"].consensus()
    ev[1].record()
    torch.cuda.synchronize()
    out = {"rank": rank, "local_nodes": plan.V, "halo_rows": len(plan.halo_nodes),
           "stored_edges": len(plan.stored_edges), "batches": len(r["rg"].batches), "vb": nb.ctx_vb,
           "mirror": nb.mirror, "z": "stored" if nb.z is not None else "derived",
           "ms_per_step": 1e3 * el / steps, "steps": steps, "consensus_ms": ev[0].elapsed_time(ev[1]) / reps,
           "exchange": exchange_model(plan, r["n_img"])}
    del r, nb, plan
    torch.cuda.empty_cache()
    return out


def proxy(name, world, t1_ms, V_total, steps, warmup):
    """proxy_8gpu entry of config ``name`` at ``world`` ranks: rank 0's share and the
    busiest rank's (if different), the exchange, the predicted speedup over one GPU."""
    ranks = sorted({0, busiest_rank(name, world)})
    shares = [time_share(name, world, r, steps, warmup) for r in ranks]
    worst = max(shares, key=lambda s: s["ms_per_step"] + s["exchange"]["ms_conservative"])
    t_c = worst["ms_per_step"] + worst["exchange"]["ms_conservative"]
    t_d = worst["ms_per_step"] + worst["exchange"]["ms_direct"]
    t_1 = worst["ms_per_step"] + worst["exchange"]["ms_one_link"]
    return {"config": name, "ranks": world, "shares": shares, "T1_ms_per_step": t1_ms,
            "per_node_cost_ratio": (worst["ms_per_step"] / worst["local_nodes"]) / (t1_ms / V_total),
            # headline prediction: the conservative exchange (one link + per-call latency)
            "predicted_ms_per_step": t_c, "predicted_speedup": t1_ms / t_c,
            "predicted_speedup_one_link": t1_ms / t_1, "predicted_speedup_direct": t1_ms / t_d}


def proxy_weak(world, value_1, steps, warmup):
    """proxy_8gpu entry of the N-GPU headline (weak scaling: ``weak8``, a ring of 8 x world
    nodes, 8 per rank): the busiest rank's share timed here plus its exchange; the predicted
    whole-job value (node-updates/s) and its ratio to the one-GPU headline ``value_1`` (C3 on
    this GPU) -- the ratio the driver's scaling run computes from its own per-N lines."""
    ranks = sorted({0, busiest_rank("weak8", world)})
    shares = [time_share("weak8", world, r, steps, warmup) for r in ranks]
    worst = max(shares, key=lambda s: s["ms_per_step"] + s["exchange"]["ms_conservative"])
    V_total = workload_cfg("weak8", world)["nodes"]
    out = {"config": "weak8", "ranks": world, "nodes": V_total, "shares": shares,
           "one_gpu_value": value_1, "scaling": "weak"}
    for tag, key in (("", "ms_conservative"), ("_one_link", "ms_one_link"), ("_direct", "ms_direct")):
        t = worst["ms_per_step"] + worst["exchange"][key]
        out[f"predicted_value{tag}"] = V_total * 1e3 / t
        out[f"predicted_speedup{tag}"] = V_total * 1e3 / t / value_1
    out["predicted_ms_per_step"] = worst["ms_per_step"] + worst["exchange"]["ms_conservative"]
    return out


def launch_ranks(n: int) -> int:
    """Run this script as ``n`` rank processes (one per GPU) and return the exit status.

    The parent has not touched the GPU (no torch import): children are started fresh with
    the torch.distributed env contract; rank 0 prints the JSON line to the shared stdout.
    If a rank fails the others are terminated (a peer blocked in a collective would hang)."""
    import signal
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 1
                print(f"bench: rank {procs.index(p)} exited with {rc}; stopping the others", file=sys.stderr)
                for q in live:
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.2)
    return status


def back_kernel_name(tr, tname, vb, mirror):
    """The batch's in-solve back projector (BACK_H = mode 3) as rocprofv3 names it: in mirror mode
    k_back_mirror_2<T, VBV, VBR> (two lane blocks per block, where the grid fills the chip) or
    k_back_mirror<T, VBV, VBR, 3>; k_back<T, VB, 3, false> otherwise.  With a traffic file, the
    one of the mirror pair that ran."""
    vbv = min(2 * vb, 32 // (8 if tname == "double" else 4))
    if not mirror:
        return f"admm::k_back<{tname}, {vb}, 3, false>"
    two = f"admm::k_back_mirror_2<{tname}, {vbv}, {vb}>"
    if tr and two in tr.get("kernels", {}):
        return two
    return f"admm::k_back_mirror<{tname}, {vbv}, {vb}, 3>"


def back_kernel_traffic(tr, tname, vb, mirror):
    """PMC bytes per launch of the batch's in-solve back projector (back_kernel_name)."""
    if not tr:
        return None
    return tr["kernels"].get(back_kernel_name(tr, tname, vb, mirror), {}).get("hbm_bytes_per_launch")


def _roof(kernel, traffic, tr_file, ms, compulsory, lds_bytes, extra=None, stale=None):
    """One kernel's roofline entry: PMC bytes per launch / live event-timed in-solve duration
    against the 8 TB/s HBM peak, compulsory bytes beside it, LDS tap reads against the
    aggregate ds_read_b128 rate.  Without a PMC file of the current kernel sources (``stale``
    says why) ``traffic`` is null and ``achieved`` falls back to the compulsory bytes."""
    s = ms * 1e-3
    basis = traffic if traffic is not None else compulsory
    roof = {
        "kernel": kernel,
        "bound": "hbm",
        "achieved": basis / s / 1e9,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": basis / s / 1e9 / HBM_PEAK_GBS,
        "traffic": traffic,
        "achieved_basis": "pmc" if traffic is not None else "compulsory",
        "traffic_source": (f"{tr_file}: rocprofv3 PMC 2 x FETCH_SIZE + WRITE_SIZE per in-solve launch "
                           "(Infinity-Cache hits included), measured on kernels of source hash "
                           f"{kernel_source_sha16()}") if traffic is not None else stale,
        "avg_launch_ms": ms,
        "compulsory_bytes": compulsory,
        "compulsory_frac": compulsory / s / 1e9 / HBM_PEAK_GBS,
        "traffic_over_compulsory": traffic / compulsory if traffic is not None else None,
        # the bound that actually applies on chip: every tap is an LDS read of a staged window
        "lds": {
            "achieved": lds_bytes / s / 1e9,
            "peak": LDS_PEAK_GBS,
            "unit": "GB/s",
            "frac": lds_bytes / s / 1e9 / LDS_PEAK_GBS,
            "bytes_per_launch": lds_bytes,
            "note": "tap reads only (staging writes excluded); peak = MI355X_MICROARCH.md aggregate "
                    "ds_read_b128 rate, all CUs streaming",
        },
    }
    roof.update(extra or {})
    assert roof["frac"] <= 1.0, roof
    return roof


def projector_rooflines(r, workload, fwd_reps):
    """Rooflines of the two projector kernels of a bound workload (each launched once per CG
    step): live HIP-event timing of their in-solve launches, PMC bytes from the committed
    passes of that workload.  Returns (dominant, forward, back, traffic, traffic file): the
    dominant one is the kernel with the larger in-solve time (both run tv x cg times)."""
    nb, geom = r["nb"], r["geom"]
    # HIP events around every CG-step launch of one more x-update each (after the timed region
    # and the halo check), each launch right after the kernel that wrote its input, as in the
    # timed steps -- the figures rocprofv3's in-solve averages must agree with; back-to-back
    # forward launches, which find the image rows still in L2, are reported beside them
    fwd_ms = nb.time_forward(in_solve=True)
    fwd_ms_warm = nb.time_forward(fwd_reps)
    back_ms = nb.time_back()
    n_img, dtype = r["n_img"], r["dtype"]
    a_node = geom.n_angles
    sb = 8 if dtype == "float64" else 4
    B_A, B_At, _ = sample_touch_bytes(n_img, a_node, TV_ITERS, CG_ITERS, sb)
    V, vb, mirror = nb.V, nb.ctx_vb, nb.mirror
    n, m = n_img * n_img, a_node * n_img
    tr, tr_file = pmc_traffic(workload)
    stale = TRAFFIC_STALE.get(workload)
    tname = "double" if dtype == "float64" else "float"
    vbv = min(2 * vb, 32 // sb)  # mirror mode's virtual width
    chunks = f"{V} nodes = {-(-V // vb)} node chunk(s) per launch"
    # forward taps: each node image read once, its sinogram written once (compulsory); the
    # design adds the transposed image copy (case-A angles) and the 8 segment partials
    fwd_comp = V * n * sb + V * m * sb
    fname = fwd_kernel_name(tr, tname, vb, mirror).replace("admm::", "").replace(" ", "")
    fwd = _roof((f"{fname} (mirror mode: virtual {vbv}-lane images over half the angles"
                 f"{'; two virtual chunks per block' if fname.endswith(',2>') else ''}; " if mirror else f"{fname} (")
                + f"Joseph forward projector taps, angle-grouped, 8 row-segment partial sums per ray; {chunks})",
                fwd_kernel_traffic(tr, tname, vb, mirror), tr_file, fwd_ms, fwd_comp,
                sb * a_node * n_img * 2 * n_img * V,  # m rays x N rows x 2 taps x V samples
                {"fwd_plan": next((dict(p) for p in nb.fwd_plans() if p["active"]), None), "mirror": mirror,
                 "avg_launch_ms_back_to_back": fwd_ms_warm,
                 "as_designed_bytes": 2 * V * n * sb + 8 * V * m * sb,
                 "sample_touch_bytes": B_A * V, "reuse_factor": B_A * V / fwd_comp,
                 "note": "frac = PMC bytes per launch / live event-timed duration of the in-solve launches "
                         "(HIP events around each CG-step forward of one x-update) / 8 TB/s. compulsory = "
                         "each node image read once + its sinogram written once. sample_touch (SURVEY 8d) "
                         "counts every tap as a load; taps are LDS reads, so it is a reuse factor, not an "
                         "HBM rate (see DESIGN.md)"}, stale)
    # back projector in H mode (A^T s fused with H p = A^T A p + rho D p + mu K^T K p and the five
    # CG dot products): compulsory = sinogram, p, D (samples) and r (float64) read once, Hp written
    back_comp = V * m * sb + 3 * V * n * sb + V * n * 8
    bname = back_kernel_name(tr, tname, vb, mirror).replace("admm::", "").replace(" ", "")
    back = _roof((f"{bname} (BACK_H; mirror mode: pixel pairs (i, j), (N-1-i, j) of the upper half over half "
                  f"the angles{'; two lane blocks per block' if 'mirror_2' in bname else ''}; " if mirror
                  else f"{bname} (BACK_H; ")
                 + f"pixel-driven Joseph adjoint taps from LDS sinogram windows, fused H epilogue and CG "
                 f"dot partials; {chunks})",
                 back_kernel_traffic(tr, tname, vb, mirror), tr_file, back_ms, back_comp,
                 sb * n * a_node * 2 * V,  # n pixels x a angles x 2 taps x V samples
                 {"mirror": mirror, "sample_touch_bytes": B_At * V,
                  "note": "frac = PMC bytes per launch / live event-timed duration of the in-solve launches "
                          "(HIP events around each CG-step back projection of one x-update) / 8 TB/s. "
                          "compulsory = sinogram, p, D read once as samples, r (float64) read once, Hp "
                          "written once"}, stale)
    dom = dict(back if back_ms >= fwd_ms else fwd)
    dom["dominant_by"] = (f"in-solve time per CG step: back {back_ms * 1e3:.1f} us vs forward taps "
                          f"{fwd_ms * 1e3:.1f} us (one launch each per CG step)")
    return dom, fwd, back, tr, tr_file


def describe(r, world):
    name = r["name"]
    if name == "weak8":
        return (f"512^2, {NODES_PER_GPU} graph nodes/GPU x {ANGLES_PER_NODE} angles (ring of {r['V_total']}; "
                f"N=2 == BASELINE configs[2]), lam=0.02 rho=2, split-Bregman {TV_ITERS}x{CG_ITERS} CG, one step "
                f"= one outer ADMM iteration")
    idx = BASELINE_INDEX.get(name)
    tag = f"BASELINE.json configs[{idx}] " if idx is not None else ""
    return (f"{name} ({tag}{r['n_img']}^2, {r['V_total']} graph nodes ({r['graph']}), {r['geom'].n_angles} "
            f"angles/node, {r['dtype']} samples, {r['tv_kind']} TV, lam=0.02 rho=2, split-Bregman "
            f"{TV_ITERS}x{CG_ITERS} CG) on {world} GPU(s), one step = one outer ADMM iteration")


def leg(name, world, rank, local_rank, steps, warmup):
    """A fixed-size config sharded over this job's ranks (strong scaling), measured."""
    import torch
    import torch.distributed as dist
    r = setup_run(name, world, rank, local_rank)
    if world > 1:
        dist.barrier()
    el = timed_steps(r, steps, max(warmup, 3), world)  # (>= 2 replays of the reuse graph before timing)
    out = {"config": name, "scaling": "strong" if name != "weak8" else "weak", "workload": describe(r, world),
           "nodes": r["V_total"], "value": r["V_total"] * steps / el, "unit": "node-updates/s",
           "ms_per_step": 1e3 * el / steps, "steps": steps, "warmup": max(warmup, 3)}
    del r
    torch.cuda.empty_cache()
    return out


def main():
    global STREAMS, EDGE_STATE
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--fwd-reps", type=int, default=20)
    ap.add_argument("--workload", choices=("auto", "C3", "weak8"), default="auto",
                    help="headline: auto = C3 on one GPU, weak8 (8 nodes per GPU) on N > 1")
    ap.add_argument("--config", choices=sorted(CONFIGS), default=None,
                    help="run a BASELINE.json config (fixed node count) instead of the headline workload")
    ap.add_argument("--as-rank", default=None, metavar="R/W",
                    help="with --config: time rank R's share of a W-rank run on this one GPU (proxy)")
    ap.add_argument("--strong", default=None,
                    help="strong-scaling configs measured after the headline, comma separated "
                         "(default: C4 on one GPU, C3,C4 on N > 1; 'none' to skip)")
    ap.add_argument("--strong-steps", type=int, default=5)
    ap.add_argument("--proxy", choices=("none", "fast", "all"), default="all",
                    help="one GPU only: per-rank proxies of the multi-GPU runs (fast: C3 on 2, C4 on 2/4/8 "
                         "ranks; all (default): + C5 on 8 ranks, which also times C5 on one GPU, and the "
                         "weak-scaling headline on 8 ranks)")
    ap.add_argument("--proxy-steps", type=int, default=6)
    ap.add_argument("--streams", type=int, default=STREAMS,
                    help="split each rank's nodes into up to this many batches (>= 8 float32 / 4 float64 "
                         "nodes each) whose kernels run concurrently on their own streams")
    ap.add_argument("--edge-state", choices=("auto", "stored", "derived"), default="auto",
                    help="z kept per edge or derived from the endpoint images (ABI 7); auto = the run's "
                         "rule (stored wherever the edge state fits, admm_hip/plan.py z_is_stored)")
    ap.add_argument("--stored-z", action="store_true", help="= --edge-state stored")
    ap.add_argument("--headline-only", action="store_true",
                    help="only the headline workload (no weak8, strong or proxy legs): rocprofv3 runs")
    args = ap.parse_args()
    if args.headline_only:
        args.strong, args.proxy = "none", "none"
    STREAMS = max(1, args.streams)
    EDGE_STATE = "stored" if args.stored_z else (None if args.edge_state == "auto" else args.edge_state)
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.as_rank is not None and args.config is None:
        ap.error("--as-rank needs --config")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))  # decided before any GPU call of this process
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        ap.error(f"--gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU, they must match")

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; ADMM_DIST_BACKEND=gloo (+ more ranks than GPUs) is a 1-GPU
    # rehearsal of the sharded path only -- the measured configuration is nccl (RCCL)
    backend = os.environ.get("ADMM_DIST_BACKEND", "nccl")
    local_rank = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)

    if args.as_rank is not None:  # one rank's share on this GPU, as its own line
        if world != 1:
            ap.error("--as-rank is a one-GPU measurement")
        R, W = (int(v) for v in args.as_rank.split("/"))
        if not (0 <= R < W):
            ap.error("--as-rank R/W needs 0 <= R < W")
        sh = time_share(args.config, W, R, args.steps, args.warmup)
        print(json.dumps({"metric": "per-rank share (proxy): ms per outer ADMM iteration", "value": sh["ms_per_step"],
                          "unit": "ms/step", "higher_is_better": False, "n_gpus": 1, "config": args.config,
                          "as_rank": args.as_rank, "share": sh}))
        return

    workload = args.config or (args.workload if args.workload != "auto" else ("C3" if world == 1 else "weak8"))
    r = setup_run(workload, world, rank, local_rank)
    if world > 1:
        dist.barrier()
    want_cpu = rank == 0 and world == 1 and not args.no_cpu_baseline and workload in ("C3", "weak8")
    first = {}

    def prime(nb):  # node 0's first x-update and its inputs, for the CPU parity check
        if want_cpu:
            first["x"] = nb.x_local[0].to("cpu").numpy().copy()
            first["b"] = nb.b[0].to("cpu").double().numpy().copy()

    el = timed_steps(r, args.steps, args.warmup, world, prime, markers=True)
    plan, geom = r["plan"], r["geom"]
    # N > 1: the halo rows the last exchange delivered (RCCL p2p / all-gather) must equal the
    # owners' images byte for byte (checked after the timed region)
    from admm_hip.exchange import verify_halo
    xcheck = verify_halo(plan, r["rg"].x_rank) if world > 1 else None
    n_img, V_total, dtype = r["n_img"], r["V_total"], r["dtype"]
    value = V_total * args.steps / el
    ms_per_step = 1e3 * el / args.steps
    roof, roof_fwd, roof_back, tr, tr_file = projector_rooflines(r, workload, args.fwd_reps)
    headline_fixed = workload in CONFIGS  # a fixed-size config (C3 headline, --config)
    result = {
        "metric": "ADMM node-updates/sec (whole node), 512² phantom; rel-Fro vs CPU ref",
        "value": value,
        "unit": "node-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if headline_fixed else "weak",
        "vs_baseline": None,
        "dtype": ("f64 samples / f64 state" if dtype == "float64" else "f32 samples / f64 state"),
        "data": "synthetic modified Shepp-Logan, on-GPU Gaussian noise sigma=0.005",
        "config": {
            "workload": describe(r, world),
            "baseline_config": BASELINE_INDEX.get(workload),
            "image": n_img, "nodes": V_total, "angles_per_node": geom.n_angles,
            "graph": r["graph"],
            "parallelism": f"graph-node shards x{world}",
            "batch_streams": len(r["rg"].streams) if r["rg"].streams else 1,
        },
        "roofline": roof,
        "roofline_fwd": roof_fwd,
        "roofline_back": roof_back,
    }
    if xcheck is not None:
        result["exchange_check"] = dict(xcheck, backend=backend, mode=r["rg"].halo.mode,
                                        ok=xcheck["mismatched_rows"] == 0)
    if tr and tr.get("per_step") and world == 1:
        sb = float(tr["per_step"]["hbm_bytes"])
        gbs = sb / (ms_per_step * 1e-3) / 1e9
        assert gbs <= HBM_PEAK_GBS, (sb, ms_per_step)
        result["step_hbm"] = {"bytes": sb, "achieved_gbs": gbs, "frac": gbs / HBM_PEAK_GBS,
                              "source": f"{tr_file} per_step (PMC, timed steps between markers)"}
    if want_cpu and "x" in first:
        result["cpu_baseline"] = cpu_baseline(n_img, geom.n_angles, first["b"], r["Wi"][0], first["x"])
    del r
    torch.cuda.empty_cache()
    if args.config:
        if rank == 0:
            print(json.dumps(result))
        if world > 1:
            dist.destroy_process_group()
        return
    # the 8-nodes-per-GPU share of the N > 1 runs, on one GPU
    if world == 1 and workload != "weak8" and not args.headline_only:
        result["weak8"] = leg("weak8", 1, 0, local_rank, args.steps, args.warmup)
    # strong scaling: fixed BASELINE configs sharded over the same ranks
    strong = args.strong if args.strong is not None else ("C4" if world == 1 else "C3,C4")
    legs = [c for c in strong.split(",") if c and c.lower() != "none"]
    result["strong"] = [leg(c, world, rank, local_rank, args.strong_steps, 1) for c in legs]
    # per-rank proxies of the multi-GPU runs (one GPU): each share timed here, exchange priced
    if world == 1 and args.proxy != "none":
        t1 = {"C3": (V_total, ms_per_step)} if workload == "C3" else {}
        for s in result["strong"]:
            t1[s["config"]] = (s["nodes"], s["ms_per_step"])
        todo = [("C3", 2), ("C4", 2), ("C4", 4), ("C4", 8)] + ([("C5", 8)] if args.proxy == "all" else [])
        px = {}
        for name, W in todo:
            if name not in t1:
                s = leg(name, 1, 0, local_rank, 2 if name == "C5" else args.strong_steps, 1)
                t1[name] = (s["nodes"], s["ms_per_step"])
            V, t = t1[name]
            px[f"{name}@{W}"] = proxy(name, W, t, V, args.proxy_steps, 1)
        if args.proxy == "all" and workload == "C3":
            px["weak8@8"] = proxy_weak(8, value, args.proxy_steps, 1)
        result["proxy_8gpu"] = dict(
            px, model=f"T_rank = rank's share timed on this GPU (halo rows fixed); exchange = bytes received "
                      f"(float64 images + statistics) over xGMI at {XGMI_LINK_GBS:.0f} GB/s per link: "
                      f"conservative = one link + {RCCL_CALL_US:.0f} us per RCCL call (assumed; 2 calls per "
                      f"iteration), one_link = one link, direct = min(peers, {XGMI_LINKS}) links; "
                      f"predicted_speedup = T_1 / (T_rank + exchange_conservative); weak8@8: predicted_value = 64 "
                      f"nodes / (T_rank + exchange), predicted_speedup = predicted_value / the one-GPU headline "
                      f"value; the rank-internal edge updates overlap the halo exchange (p2p or all-gather; "
                      f"not priced)")
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
