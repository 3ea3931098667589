"""Benchmark: decentralized-ADMM node-updates/s on MI355X (BASELINE.json metric).

Workload (weak scaling, one process per GPU): 512^2 modified Shepp-Logan,
8 graph nodes per GPU with 96 angles each (N GPUs -> 8N-node ring; N=2 is
BASELINE configs[2] exactly: 16 nodes, 1536 angles = 3N), lambda_TV = 0.02,
rho = 2, split-Bregman 10 rounds x 5 CG steps per x-update, float32 projector
samples / float64 solver state.  A "step" is one outer ADMM iteration: the
x-update of every node, the halo exchange (RCCL), the z/y edge updates and the
residual/statistics readback the reference's stop test needs.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...
    python bench.py --config C2|C3|C4|C5     (BASELINE.json configs[1..4], fixed node count,
                                               sharded over however many ranks run it)

Rank 0 prints one JSON line.  The forward projector's average launch time is
measured live with HIP events on the stream it runs on; its algorithmic
(sample-touch) bytes are B_A = 4 m (2N+1) per node.  The CPU
baseline is the float64 NumPy/SciPy oracle (oracle/, a port of the reference
algorithm; the reference's CVXPY/ODL path cannot run here) timed on a bounded
sample of the same workload on rank 0's host cores.
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
NODES_PER_GPU = 8
ANGLES_PER_NODE = 96
LAM, RHO = 0.02, 2.0
TV_ITERS, CG_ITERS = 10, 5
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
LDS_PEAK_GBS = 150000.0  # aggregate ds_read_b128 rate, every CU streaming (MI355X_MICROARCH.md, LDS)


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


def node_bytes(N, a, tv, cg, sample_bytes=4):
    """Algorithmic sample-touch bytes of one x-update (4-byte samples, 8 in C5)."""
    m = a * N
    n = N * N
    sb = sample_bytes
    B_A = sb * m * (2 * N + 1)
    B_At = sb * n * (2 * a + 1)
    B_cg = B_A + B_At + 6 * sb * n + 14 * sb * n
    return B_A, B_At, tv * (cg * B_cg + 27 * sb * n) + B_At + sb * n * (3 * 2 + 2)


def cpu_baseline(seconds_budget=20.0):
    """Oracle (float64 NumPy/SciPy) x-updates at the bench size on this host."""
    import numpy as np
    from oracle import node_solver as ons
    from oracle.geometry import Geometry, joseph_matrix, shepp_logan
    t0 = time.perf_counter()
    A = joseph_matrix(Geometry(N_IMG, ANGLES_PER_NODE))
    AT = A.T.tocsr()
    build_s = time.perf_counter() - t0
    x_true = shepp_logan(N_IMG, 2).ravel()
    b = A @ x_true + 0.005 * np.random.default_rng(1000).standard_normal(A.shape[0])
    W = np.maximum(np.asarray(A.multiply(A).sum(axis=0)).ravel(), 1e-12)
    q = W  # arithmetic mean of identical W
    Atb = AT @ b
    prm = ons.NodeParams(rho=RHO, lam=LAM, mu=10 * LAM, tv_iters=TV_ITERS, cg_iters=CG_ITERS)
    n = N_IMG * N_IMG
    st = ons.NodeState.zeros(n)
    v = np.zeros(n)
    done = 0
    t0 = time.perf_counter()
    while True:
        ons.node_update(A, Atb, b, 2 * q, 2 * q * v, [(q, v), (q, v)], st, N_IMG, prm, AT=AT)
        done += 1
        el = time.perf_counter() - t0
        if el > seconds_budget or done >= 3:
            break
    return {"value": done / el, "unit": "node-updates/s", "cores": 1, "kind": "port",
            "sample": f"{done} x-update(s) of one 512^2 node (96 angles, 2 ring neighbours, "
                      f"10x5 inner), float64 SciPy CSR Joseph matrix, single thread; "
                      f"{el:.1f} s timed, {build_s:.1f} s matrix build excluded"}


# HBM bytes per forward-projector launch from the committed rocprofv3 PMC summary
# (scripts/pmc.sh + scripts/traffic_summary.py; 2 x FETCH_SIZE + WRITE_SIZE per the
# MI355X_MICROARCH.md gfx950 correction).  PMC counters cannot be read inside this run.
TRAFFIC_FILE = "profiles/r1_traffic.json"
FWD_KERNELS = ("admm::k_fwdg<float, 8>",)


def pmc_traffic(names):
    try:
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), TRAFFIC_FILE)) as f:
            k = json.load(f)["kernels"]
        return float(sum(k[n]["hbm_bytes_per_launch"] for n in names))
    except (OSError, KeyError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--fwd-reps", type=int, default=20)
    ap.add_argument("--config", choices=sorted(CONFIGS), default=None,
                    help="run a BASELINE.json config (fixed node count) instead of the default workload")
    args = ap.parse_args()

    import networkx as nx
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
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

    from admm_hip.data import make_precisions, make_sinograms, shepp_logan
    from admm_hip.exchange import HaloExchange, assemble_stats
    from admm_hip.plan import make_plan
    from admm_hip.solver import NodeBatch, make_operators

    if args.config:
        cfg = CONFIGS[args.config]
        n_img, V_total, dtype, tv_kind = cfg["N"], cfg["nodes"], cfg["dtype"], cfg["tv"]
        G = make_graph(cfg["graph"], V_total)
        angles_total = max(180, 3 * n_img)  # block_2_load_odl_data.py:31-38
        if "angles_per_node" in cfg:  # a share of a larger config keeps its per-node angle count
            angles_total = cfg["angles_per_node"] * V_total
    else:
        n_img, V_total, dtype, tv_kind = N_IMG, NODES_PER_GPU * world, "float32", "iso"
        G = nx.cycle_graph(V_total)
        angles_total = ANGLES_PER_NODE * V_total
    ops = make_operators(n_img, V_total, angles_total=angles_total, dtype=dtype, device=local_rank)
    geom = ops[0].geom
    plan = make_plan(G, V_total, world, rank)
    ph = shepp_logan(n_img)
    lo = plan.local_nodes[0]
    sinos = dict(zip(plan.local_nodes,
                     make_sinograms([ops[g] for g in plan.local_nodes], ph, 0.005, seed=1000 + lo)))
    Wi, Q = make_precisions(ops)  # one W kernel launch: every node shares the geometry
    nb = NodeBatch(geom, dtype, plan, sinos, Q, RHO, LAM, 10 * LAM, TV_ITERS, CG_ITERS, tv_kind,
                   ph, local_rank, keep_x=True)
    halo = HaloExchange(plan, nb.x_ext)
    if world > 1:
        dist.barrier()

    def step():
        nb.node_update()
        halo.run()
        nb.consensus()
        return assemble_stats(plan, nb.node_stats, nb.edge_stats[: len(plan.stored_edges)])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ns, es = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    value = V_total * args.steps / el

    # live measurement of the dominant kernel (forward projector) on its stream
    fwd_ms = nb.time_forward(args.fwd_reps)
    a_node = geom.n_angles
    sbytes = 8 if dtype == "float64" else 4
    B_A, B_At, B_node = node_bytes(n_img, a_node, TV_ITERS, CG_ITERS, sbytes)
    achieved = B_A * plan.V / (fwd_ms * 1e-3) / 1e9
    lds_bytes = sbytes * a_node * n_img * 2 * n_img * plan.V  # m rays x N rows x 2 taps x V samples
    fwd_traffic = pmc_traffic(FWD_KERNELS) if not args.config else None
    if args.config:
        workload = (f"{args.config}: {n_img}^2, {V_total} graph nodes ({CONFIGS[args.config]['graph']}), "
                    f"{a_node} angles/node, {dtype} samples, {tv_kind} TV, lam=0.02 rho=2, split-Bregman "
                    f"{TV_ITERS}x{CG_ITERS} CG, one step = one outer ADMM iteration")
    else:
        workload = (f"512^2, {NODES_PER_GPU} graph nodes/GPU x {ANGLES_PER_NODE} angles (ring of "
                    f"{V_total}; N=2 == BASELINE configs[2]), lam=0.02 rho=2, split-Bregman "
                    f"{TV_ITERS}x{CG_ITERS} CG, one step = one outer ADMM iteration")
    result = {
        "metric": "ADMM node-updates/sec (whole node), 512² phantom; rel-Fro vs CPU ref",
        "value": value,
        "unit": "node-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * el / args.steps,
        "higher_is_better": True,
        "scaling": "strong" if args.config else "weak",
        "vs_baseline": None,
        "dtype": ("f64 samples / f64 state" if dtype == "float64" else "f32 samples / f64 state"),
        "data": "synthetic modified Shepp-Logan, on-GPU Gaussian noise sigma=0.005",
        "config": {
            "workload": workload,
            "image": n_img, "nodes": V_total, "angles_per_node": a_node,
            "graph": CONFIGS[args.config]["graph"] if args.config else "ring",
            "parallelism": f"graph-node shards x{world}",
        },
        "roofline": {
            "kernel": f"k_fwdg<{'double' if dtype == 'float64' else 'float'},{nb.ctx_vb}> (Joseph forward "
                      "projector taps, angle-grouped; its 8-segment partial sums are added by "
                      "k_fwd_combine, ~5 us at 512^2, not included)",
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": fwd_traffic,
            "traffic_source": TRAFFIC_FILE if fwd_traffic is not None else None,
            # measured DRAM rate of the same launch: PMC bytes / event-timed duration
            "traffic_gbs": fwd_traffic / (fwd_ms * 1e-3) / 1e9 if fwd_traffic is not None else None,
            "avg_launch_ms": fwd_ms,
            "bytes_per_launch": B_A * plan.V,
            "note": "sample-touch bytes (SURVEY 8d); image/sinogram are L2/MALL resident, so frac>1 "
                    "means on-chip reuse, see DESIGN.md",
            # the bound that actually applies on chip: every tap is an LDS read of the staged
            # window (2 taps x V samples per ray and row), against the measured ds_read_b128 peak
            "lds": {
                "achieved": lds_bytes / (fwd_ms * 1e-3) / 1e9,
                "peak": LDS_PEAK_GBS,
                "unit": "GB/s",
                "frac": lds_bytes / (fwd_ms * 1e-3) / 1e9 / LDS_PEAK_GBS,
                "bytes_per_launch": lds_bytes,
                "note": "tap reads only (staging writes excluded); peak = MI355X_MICROARCH.md aggregate "
                        "ds_read_b128 rate, all CUs streaming",
            },
        },
        "node_update_bytes": B_node,
        "node_update_gbs": B_node * value / world / 1e9,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.config:
        result["cpu_baseline"] = cpu_baseline()
        result["cpu_baseline"]["cores"] = 1
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
