"""CPU: graph-node sharding plan, and the N>1 path (halo exchange + deterministic
statistics) on world_size-2 gloo with CPU tensors.

The sharded run below drives the *product* plan/exchange code with the CPU
oracle standing in for the device kernels, and must reproduce the
single-process oracle trajectory bitwise (1-GPU vs N-GPU
trajectory equality).
"""
import math
import os
import socket

import networkx as nx
import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from admm_hip.plan import make_plan, node_ranges


def graphs():
    yield "ring8", nx.cycle_graph(8)
    yield "path5", nx.path_graph(5)
    yield "complete6", nx.complete_graph(6)
    seed = next(s for s in range(100) if nx.is_connected(nx.erdos_renyi_graph(9, 0.35, seed=s)))
    yield "er9", nx.erdos_renyi_graph(9, 0.35, seed=seed)


def scale_graphs():
    """The graphs the 8-GPU runs use: the bench's default workload at N = 8 (a ring of 64),
    C4's 32-node Erdos-Renyi graph (committed fixture) and C5's 64-node complete graph."""
    import json
    yield "ring64", nx.cycle_graph(64)
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c4_er32_graph.json")) as f:
        fx = json.load(f)
    G = nx.Graph()
    G.add_nodes_from(range(fx["nodes"]))
    G.add_edges_from(map(tuple, fx["edges"]))
    yield "er32", G
    yield "complete64", nx.complete_graph(64)


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_exchange_mode_is_the_same_on_every_rank(world):
    """HaloExchange is a collective: p2p or all-gather must be one global choice.  C4's
    ER graph on 8 ranks has ranks on both sides of the per-rank density threshold."""
    for name, G in list(graphs()) + list(scale_graphs()):
        V = G.number_of_nodes()
        if V < world:
            continue
        modes = {make_plan(G, V, world, r).use_allgather() for r in range(world)}
        assert len(modes) == 1, (name, world)
    # the byte-minimising rule: ER graphs exchange halo rows point to point (C4@8: at most 21
    # halo rows against 28 all-gathered images), complete graphs all-gather
    G = dict(scale_graphs())["er32"]
    assert not make_plan(G, 32, 8, 0).use_allgather()
    assert make_plan(nx.complete_graph(64), 64, 8, 0).use_allgather()


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_exchange_mode_minimises_the_busiest_ranks_bytes(world):
    """The chosen halo exchange lands no more images on the busiest rank than the other mode
    would: all-gather (world - 1) x vmax per rank, p2p a rank's halo rows."""
    for name, G in list(graphs()) + list(scale_graphs()):
        V = G.number_of_nodes()
        if V < world:
            continue
        plans = [make_plan(G, V, world, r) for r in range(world)]
        vmax = max(hi - lo for lo, hi in plans[0].ranges)
        ag, p2p = (world - 1) * vmax, max(len(p.halo_nodes) for p in plans)
        chosen = ag if plans[0].use_allgather() else p2p
        assert chosen <= min(ag, p2p), (name, world, ag, p2p)


@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_plan_partitions_nodes_and_edges(world):
    for name, G in graphs():
        V = G.number_of_nodes()
        plans = [make_plan(G, V, world, r) for r in range(world)]
        # nodes: contiguous, disjoint, complete
        allnodes = sum((p.local_nodes for p in plans), [])
        assert allnodes == list(range(V)), name
        # every edge is owned exactly once, stored by both endpoint owners
        owned = {}
        for p in plans:
            for k, ge in enumerate(p.stored_edges):
                if p.owned_edge[k]:
                    assert ge not in owned
                    owned[ge] = p.rank
        assert sorted(owned) == list(range(len(p.edges)))
        for p in plans:
            loc = set(p.local_nodes)
            for ge, (a, b) in enumerate(p.edges):
                assert (ge in p.stored_edges) == (a in loc or b in loc)
            # halo = remote neighbours
            halo = {j for i in p.local_nodes for j in G.neighbors(i)} - loc
            assert set(p.halo_nodes) == halo
            # incidence in G.neighbors order with the right sign
            for k, g in enumerate(p.local_nodes):
                nbrs = [p.inc_nbr[q] for q in range(p.inc_off[k], p.inc_off[k + 1])]
                assert nbrs == list(G.neighbors(g))
                for q in range(p.inc_off[k], p.inc_off[k + 1]):
                    a, b = p.edges[p.stored_edges[p.inc_edge[q]]]
                    assert p.inc_sign[q] == (1 if g == a else -1)
            # send/recv plans are mutually consistent
            for peer, nodes in p.send.items():
                assert plans[peer].recv[p.rank] == nodes


def test_node_ranges_balanced():
    for V in range(1, 20):
        for W in range(1, 9):
            r = node_ranges(V, W)
            sizes = [hi - lo for lo, hi in r]
            assert sum(sizes) == V and max(sizes) - min(sizes) <= 1


def test_allgather_choice():
    assert not make_plan(nx.cycle_graph(16), 16, 2, 0).use_allgather()
    assert make_plan(nx.complete_graph(16), 16, 2, 0).use_allgather()


# ----------------------------------------------------------------------------
# world_size 2, gloo, CPU tensors
# ----------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sharded_oracle_admm(rank, world, port, gname, out_q, overlap=False):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(os.path.dirname(here), "distributed-inverse-problem-admm_amd"),
              os.path.dirname(here)):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from admm_hip.exchange import HaloExchange, assemble_stats, gather_images
        from admm_hip.plan import make_plan
        res = run_sharded(rank, world, gname, HaloExchange, assemble_stats, gather_images, make_plan, overlap)
        out_q.put((rank, res))
    finally:
        dist.destroy_process_group()


def problem(gname):
    from oracle.geometry import Geometry, joseph_matrix, shepp_logan
    G = dict(graphs())[gname]
    V = G.number_of_nodes()
    N = 12
    A = joseph_matrix(Geometry(N, 9))
    ph = shepp_logan(N, 2).ravel()
    sinos = [A @ ph + 0.01 * np.random.default_rng(i).standard_normal(A.shape[0]) for i in range(V)]
    W = np.maximum(np.asarray(A.multiply(A).sum(axis=0)).ravel(), 1e-12)
    return G, V, N, A, ph, sinos, W


def test_subset_plans_of_operator_groups():
    """Groups of one rank's nodes (admm_hip/groups.py): every group holds every edge incident
    to it, each edge is owned by exactly one group (the one with its lower endpoint), halo
    rows are exactly the out-of-group neighbours, and incidence lists keep G.neighbors order."""
    from admm_hip.plan import make_plan, make_subset_plan
    G = nx.erdos_renyi_graph(12, 0.4, seed=3)
    rp = make_plan(G, 12, 2, 1)  # nodes 6..11
    groups = [[6, 8, 9], [7, 11], [10]]
    plans = [make_subset_plan(G, 12, g, 2, 1, rp.ranges, rp.edges) for g in groups]
    owned = {}
    for P, g in zip(plans, groups):
        assert P.local_nodes == sorted(g)
        nb = {j for i in g for j in G.neighbors(i)} - set(g)
        assert P.halo_nodes == sorted(nb)
        for k, ge in enumerate(P.stored_edges):
            a, b = P.edges[ge]
            assert a in g or b in g
            assert P.edge_a_row[k] == P.xrow[a] and P.edge_b_row[k] == P.xrow[b]
            if P.owned_edge[k]:
                assert ge not in owned and a in g
                owned[ge] = True
        for k, i in enumerate(P.local_nodes):
            nbrs = [P.inc_nbr[q] for q in range(P.inc_off[k], P.inc_off[k + 1])]
            assert nbrs == list(G.neighbors(i))
    # together the groups own exactly the edges the rank plan owns
    assert sorted(owned) == sorted(ge for k, ge in enumerate(rp.stored_edges) if rp.owned_edge[k])


def run_sharded(rank, world, gname, HaloExchange, assemble_stats, gather_images, make_plan, overlap=False):
    """The device loop of admm_hip.admm.run_admm with the oracle in place of the kernels.
    ``overlap``: RankGroups.exchange_consensus's order -- the exchange issued asynchronously
    (HaloExchange.start), the internal edge slots [0, n_internal) updated from the local rows
    while it is in flight, then the halo rows landed (finish) and the remaining slots updated."""
    from oracle import node_solver as ons
    G, V, N, A, ph, sinos, W = problem(gname)
    n = N * N
    rho, lam = 2.0, 0.02
    prm = ons.NodeParams(rho=rho, lam=lam, mu=10 * lam, tv_iters=2, cg_iters=3)
    plan = make_plan(G, V, world, rank)
    x_ext = torch.zeros((plan.n_xext, n), dtype=torch.float64)
    E = len(plan.stored_edges)
    y = np.zeros((E, n))
    z = np.zeros((E, n))
    states = {g: ons.NodeState.zeros(n) for g in plan.local_nodes}
    halo = HaloExchange(plan, x_ext)
    hist = {"primal": [], "dual": [], "obj": []}
    for k in range(3):
        node_stats = torch.zeros((plan.V, 6), dtype=torch.float64)
        for r, g in enumerate(plan.local_nodes):
            D = np.zeros(n)
            c = np.zeros(n)
            qv = []
            for q in range(plan.inc_off[r], plan.inc_off[r + 1]):
                e = plan.inc_edge[q]
                v = z[e] - plan.inc_sign[q] * y[e]
                D += W
                c += W * v
                qv.append((W, v))
            d = ons.node_update(A, A.T @ sinos[g], sinos[g], D, c, qv, states[g], N, prm)
            x_ext[r] = torch.from_numpy(states[g].x)
            node_stats[r] = torch.tensor([d.mse_sino, d.g_norm ** 2, d.tv, d.quad, 0.0, d.sb_res ** 2])
        edge_stats = torch.zeros((max(E, 1), 3), dtype=torch.float64)

        def edges(s0, s1, rows):
            xs = x_ext[:rows].numpy()
            for s in range(s0, s1):
                ra, rb = plan.edge_a_row[s], plan.edge_b_row[s]
                assert ra < rows and rb < rows
                xa, xb = xs[ra], xs[rb]
                aa, ab = xa + y[s], xb - y[s]
                zn = (aa + ab) * 0.5
                y[s] = y[s] + xa - zn
                dz = zn - z[s]
                z[s] = zn
                edge_stats[s] = torch.tensor([float((xa - zn) @ (xa - zn)), float((xb - zn) @ (xb - zn)),
                                              float(dz @ dz)])
        if overlap:
            h = halo.start()
            edges(0, plan.n_internal, plan.V)  # both endpoints local: rows < V
            halo.finish(h)
            edges(plan.n_internal, E, plan.n_xext)
        else:
            halo.run()
            edges(0, E, plan.n_xext)
        ns, es = assemble_stats(plan, node_stats, edge_stats[:E])
        r2 = sum(float(es[ge, 0]) + float(es[ge, 1]) for ge in range(len(plan.edges)))
        s2 = sum(rho * rho * float(es[ge, 2]) for ge in range(len(plan.edges)))
        hist["primal"].append(math.sqrt(r2))
        hist["dual"].append(math.sqrt(s2))
        hist["obj"].append(ns[:, 0].numpy().copy())
    X = gather_images(plan, x_ext[: plan.V])
    return X.numpy().copy(), hist


# world 2: both halo directions go to the same peer; world 4 on the ring: distinct left and
# right peers (the 8-GPU layout), on the ER graph an uneven 3/2/2/2 split with p2p to several
# peers; the complete graph all-gathers
@pytest.mark.parametrize("gname,world", [("ring8", 2), ("complete6", 2), ("er9", 2), ("ring8", 4), ("er9", 4)])
def test_gloo_sharded_matches_single_process_bitwise(gname, world):
    from admm_hip.exchange import HaloExchange, assemble_stats, gather_images
    X1, h1 = run_sharded(0, 1, gname, HaloExchange, assemble_stats, gather_images, make_plan)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_oracle_admm, args=(r, world, port, gname, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        X2, h2 = res[r]
        assert np.array_equal(X1, X2), gname
        assert h1["primal"] == h2["primal"] and h1["dual"] == h2["dual"], gname
        for a, b in zip(h1["obj"], h2["obj"]):
            assert np.array_equal(a, b)
    # the oracle's own (unsharded) loop agrees with the plan-driven loop to rounding
    # (it applies A^T through a CSR copy, so its sums run in a different order)
    from oracle import admm as oadmm
    G, V, N, A, ph, sinos, W = problem(gname)
    xo, ho = oadmm.decentralized_admm([A] * V, sinos, G, lambda i, j: W, N, lam_tv=0.02, rho=2.0,
                                      max_iters=3, eps_pri=0.0, eps_dual=0.0, tv_iters=2, cg_iters=3)
    assert np.abs(np.stack(xo) - X1).max() <= 1e-10 * np.abs(X1).max()
    assert np.allclose(ho["primal"], h1["primal"], rtol=1e-7, atol=0)
    assert np.allclose(ho["dual"], h1["dual"], rtol=1e-7, atol=0)


@pytest.mark.parametrize("gname,world", [("er9", 4), ("ring8", 4), ("complete6", 2)])
def test_gloo_overlapped_exchange_matches_serial_bitwise(gname, world):
    """RankGroups.exchange_consensus's order (rank-internal edges updated while the halo images
    are in flight: asynchronous all-gather on the complete graph, p2p on the ring and ER) gives the
    serial exchange-then-consensus run bitwise, and the single-process run."""
    from admm_hip.exchange import HaloExchange, assemble_stats, gather_images
    X1, h1 = run_sharded(0, 1, gname, HaloExchange, assemble_stats, gather_images, make_plan)
    # internal edges (some rank has them to overlap) come first in slot order
    G = dict(graphs())[gname]
    assert any(make_plan(G, G.number_of_nodes(), world, r).n_internal for r in range(world))
    for r in range(world):
        p = make_plan(G, G.number_of_nodes(), world, r)
        assert all(p.edge_a_row[k] < p.V and p.edge_b_row[k] < p.V for k in range(p.n_internal))
        assert all(max(p.edge_a_row[k], p.edge_b_row[k]) >= p.V for k in range(p.n_internal, len(p.stored_edges)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_oracle_admm, args=(r, world, port, gname, q, True)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        X2, h2 = res[r]
        assert np.array_equal(X1, X2), gname
        assert h1["primal"] == h2["primal"] and h1["dual"] == h2["dual"], gname


def _placement_rank(rank, world, port, q):
    """INTEGRATION.md's recipe on a rank: torch.cuda.set_device(local_rank) before building
    anything.  No GPU here, so the current-device query stands in for it (monkeypatched
    per rank); only host-side construction runs (operators are lazy, nothing launches)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.is_available = lambda: True
        torch.cuda.current_device = lambda: rank  # what set_device(local_rank) leaves behind
        from admm_hip.geometry import ParallelBeamGeometry, RayTransform
        from admm_hip.solver import make_operators
        ops = make_operators(64, 4)
        one = RayTransform(ParallelBeamGeometry(64, 45))
        q.put((rank, [A.device for A in ops] + [one.device, one.T.device]))
    finally:
        dist.destroy_process_group()


def test_operators_follow_each_ranks_current_device():
    """Operators default to the caller's current device, so N ranks after
    torch.cuda.set_device(local_rank) build on N different GPUs (not all on GPU 0)."""
    import inspect
    import block_2_load_odl_data
    from admm_hip.geometry import RayTransform
    from admm_hip.solver import make_operators
    assert inspect.signature(make_operators).parameters["device"].default is None
    assert inspect.signature(RayTransform).parameters["device"].default is None
    assert inspect.signature(block_2_load_odl_data.load_odl_data).parameters["device"].default is None
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_placement_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == {0: [0] * 6, 1: [1] * 6}


def _halo_check_rank(rank, world, port, gname, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "distributed-inverse-problem-admm_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from admm_hip.exchange import HaloExchange, verify_halo
        G = dict(list(graphs()) + list(scale_graphs()))[gname]
        V = G.number_of_nodes()
        plan = make_plan(G, V, world, rank)
        n = 37
        x = torch.zeros((plan.n_xext, n), dtype=torch.float64)
        for g in plan.local_nodes:  # node g's image: a function of g only
            x[plan.xrow[g]] = torch.from_numpy(np.random.default_rng(g).standard_normal(n))
        before = verify_halo(plan, x)  # halo rows still zero
        HaloExchange(plan, x).run()
        after = verify_halo(plan, x)
        if plan.halo_nodes:  # one flipped bit in one halo row
            x[plan.xrow[plan.halo_nodes[0]]].view(torch.int64)[3] ^= 1
        flipped = verify_halo(plan, x)
        q.put((rank, (before, after, flipped, len(plan.halo_nodes))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("gname,world", [("ring8", 2), ("complete6", 2), ("ring8", 4), ("ring64", 8),
                                         ("er32", 8), ("complete64", 8)])
def test_verify_halo_detects_exchange_errors(gname, world):
    """bench.py's N > 1 exchange check (admm_hip.exchange.verify_halo): after HaloExchange.run
    every halo row equals its owner's row byte for byte; before it, or with one bit
    flipped, the check reports the rows."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_halo_check_rank, args=(r, world, port, gname, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    total = sum(res[r][3] for r in range(world))
    flips = sum(1 for r in range(world) if res[r][3])
    for r in range(world):
        before, after, flipped, _ = res[r]
        assert before == {"halo_rows": total, "mismatched_rows": total}
        assert after == {"halo_rows": total, "mismatched_rows": 0}
        assert flipped == {"halo_rows": total, "mismatched_rows": flips}


# ---------------------------------------------------------------------------------------
# the run's one edge-state rule (stored vs derived z; plan.z_is_stored, groups.py)
# ---------------------------------------------------------------------------------------
class _Op:
    """Host stand-in of a RayTransform for the batch-grouping logic (operator_key)."""

    def __init__(self, N, a, dtype="float32"):
        from admm_hip.geometry import ParallelBeamGeometry
        self.geom = ParallelBeamGeometry(N, a)
        self.dtype = dtype
        self.device = 0


HBM_MI355X = 288 * 10**9


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_stored_z_for_every_baseline_config_at_every_gpu_count(world):
    """C3 (16-node ring, 512^2), C4 (32-node ER, 1024^2), C5 (64-node complete,
    2048^2, float64): the stored edge state (y, z) of the busiest rank fits the rule's share of 288 GB
    at 1, 2, 4 and 8 GPUs -- stored z (faster, profiles/r4_shares_derived_vs_stored_z.txt)
    everywhere, so one problem runs the same edge arithmetic at every GPU count (the 1-rank
    vs N-rank bitwise tests need that)."""
    from admm_hip.groups import stored_edges_per_rank
    from admm_hip.plan import z_is_stored
    sg = dict(scale_graphs())
    cases = [("C3", nx.cycle_graph(16), 16, 512, "float32"), ("C4", sg["er32"], 32, 1024, "float32"),
             ("C5", sg["complete64"], 64, 2048, "float64")]
    for name, G, V, N, dt in cases:
        ops = [_Op(N, 96, dt)] * V
        per = stored_edges_per_rank(ops, G, V, world)
        assert len(per) == world
        assert z_is_stored(per, N * N, HBM_MI355X), (name, world, per)
    # C5 on one GPU is two batches (56 + 8 nodes: 32-bit offsets), the cross edges stored twice
    assert stored_edges_per_rank([_Op(2048, 96, "float64")] * 64, sg["complete64"], 64, 1) == [2464]


def test_derived_z_when_stored_would_not_fit():
    """A graph whose stored edge state exceeds the rule's share of HBM derives z (weighted
    fusion never)."""
    from admm_hip.groups import stored_edges_per_rank
    from admm_hip.plan import STORED_Z_HBM_FRACTION, stored_edge_state_bytes, z_is_stored
    G = nx.complete_graph(48)
    per = stored_edges_per_rank([_Op(2048, 96, "float64")] * 48, G, 48, 1)
    assert per == [48 * 47 // 2]
    hbm = int(stored_edge_state_bytes(per, 2048 * 2048) / STORED_Z_HBM_FRACTION) - 1
    assert not z_is_stored(per, 2048 * 2048, hbm)
    assert z_is_stored(per, 2048 * 2048, hbm + 1)
    assert z_is_stored(per, 2048 * 2048, hbm, fusion="weighted")


def _z_rule_rank(rank, world, port, hbm, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from admm_hip.groups import min_over_ranks, stored_edges_per_rank
        from admm_hip.plan import z_is_stored
        # every rank weighs the same global inputs; the device HBM is agreed by one MIN all-reduce
        # (rank 1 here reports a smaller device, so the agreed HBM derives z on every rank)
        G = nx.complete_graph(48)
        per = stored_edges_per_rank([_Op(2048, 96, "float64")] * 48, G, 48, world)
        agreed = min_over_ranks(hbm[rank], world)
        q.put((rank, agreed, z_is_stored(per, 2048 * 2048, agreed)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_z_rule_same_answer_on_every_rank(world):
    """The rule is one global decision: with per-rank device HBM that differs (rank 1 smaller,
    below the C5-like graph's threshold), every rank of a gloo world 2 / 4 / 8 gets the same
    HBM from the MIN all-reduce and the same stored / derived answer."""
    from admm_hip.groups import stored_edges_per_rank
    from admm_hip.plan import STORED_Z_HBM_FRACTION, stored_edge_state_bytes
    per = stored_edges_per_rank([_Op(2048, 96, "float64")] * 48, nx.complete_graph(48), 48, world)
    need = int(stored_edge_state_bytes(per, 2048 * 2048) / STORED_Z_HBM_FRACTION)
    hbm = [need + 10**9] * world
    hbm[1] = need - 10**9
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_z_rule_rank, args=(r, world, port, hbm, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert {r[1] for r in res} == {need - 10**9}
    assert {r[2] for r in res} == {False}
