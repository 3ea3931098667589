"""GPU: the sharded product path (NodeBatch + HaloExchange + assemble_stats +
gather_images) with 2 ranks sharing one GPU over gloo, against 1 rank.

The real configuration is one rank per GPU over RCCL; this runs the same
kernels and plan/exchange code with gloo (host-staged copies) so the N>1 path
is exercised on the device in a 1-GPU session.  Trajectories and images must
be bitwise identical to the single-rank run.  The "unequal" case
splits 100 angles over 6 nodes (17,17,17,17,16,16: the reference's own remainder rule,
block_2_load_odl_data.py:35-38), so nodes with different operators run as separate device
batches (admm_hip/groups.py) within a rank as well as across ranks.
"""
import os
import socket

import networkx as nx
import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem(angles=96):
    import sys
    for p in (os.path.join(ROOT, "distributed-inverse-problem-admm_amd"), ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    from admm_hip.data import make_precisions, make_sinograms, shepp_logan
    from admm_hip.solver import make_operators
    N, V = 40, 6
    ops = make_operators(N, V, angles, device=0)
    ph = shepp_logan(N)
    sinos = make_sinograms(ops, ph, 0.005, seed=1000)
    Wi, Q = make_precisions(ops)
    return N, V, ops, ph, sinos, Wi, Q


def _run(graph, fusion, angles=96, group=None):
    from block_6_admm_loop_ver2 import decentralized_admm
    N, V, ops, ph, sinos, Wi, Q = _problem(angles)
    G = {"ring": nx.cycle_graph(V), "complete": nx.complete_graph(V)}[graph]
    if fusion == "weighted":
        rng = np.random.default_rng(2)
        Wi = [np.asarray(w) * np.exp(0.5 * rng.standard_normal(N * N)) for w in Wi]
    x, h = decentralized_admm(ops, sinos, G, Wi, Q, N, lam_tv=0.02, rho=2.0, max_iters=4, eps_pri=0.0,
                              eps_dual=0.0, verbose=False, phantom_true=ph, write_params=False,
                              group=group, fusion=fusion)
    return np.stack(x), {k: np.asarray(h[k]) for k in ("primal", "dual", "obj_total", "mse_sino_total")}


def _worker(rank, world, port, graph, fusion, angles, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, _run(graph, fusion, angles)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("graph,fusion,angles", [("ring", "midpoint", 96), ("complete", "weighted", 96),
                                                ("complete", "midpoint", 100), ("ring", "weighted", 100)],
                         ids=["ring", "complete-weighted", "unequal-complete", "unequal-ring-weighted"])
def test_two_ranks_on_one_gpu_match_one_rank_bitwise(cuda, graph, fusion, angles):
    x1, h1 = _run(graph, fusion, angles)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, graph, fusion, angles, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for r in range(2):
        x2, h2 = res[r]
        assert np.array_equal(x1, x2), (graph, fusion, r)
        for k in h1:
            assert np.array_equal(h1[k], h2[k]), (k, graph, fusion)


@pytest.mark.timeout(180)
def test_rccl_calls_on_one_rank(cuda):
    """The RCCL calls of the multi-GPU path on a one-rank "nccl" group (scripts/probes/
    rccl_one_gpu.py, its own process): all_gather_into_tensor of float64 device rows (async),
    a grouped batch_isend_irecv into a row slice (to the rank itself), all_reduce SUM / MAX of
    float64 and int64 device tensors, barrier.  RCCL refuses two ranks on one GPU, so the
    cross-rank semantics are covered by the gloo tests; this pins the call signatures, dtypes and
    views on RCCL itself."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = socket.socket()
    port.bind(("127.0.0.1", 0))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port.getsockname()[1]))
    port.close()
    p = subprocess.run([sys.executable, os.path.join(root, "scripts", "probes", "rccl_one_gpu.py")],
                       env=env, capture_output=True, text=True, timeout=150)
    print(p.stdout[-400:])
    assert p.returncode == 0, p.stderr[-2000:]
    assert "'all_gather_into_tensor': True" in p.stdout and "'batch_isend_irecv_self': True" in p.stdout
