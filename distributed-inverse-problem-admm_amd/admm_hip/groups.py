"""One rank's graph nodes as device batches, one batch per distinct operator.

The batched kernels project every node of a batch with one angle table (or one CSR
matrix): node-interleaved samples put the same pixel of VB nodes in one vector, so
those nodes must share A.  The reference does not guarantee that: ``load_odl_data``
splits ``max(180, 3N)`` angles over the nodes with the remainder going to the first
ones (/root/reference/block_2_load_odl_data.py:31-38) -- its own defaults give
77/77/77/77/76 angles at N=128 and 39/39/38/38/38 at N=64 with 5 nodes
(block_7_main_ver3.py:334-335) -- and a saved ``A_dense_list`` may hold any matrices.

``RankGroups`` therefore splits the rank's nodes by operator key (geometry or matrix
digest, sample dtype, device) into node batches (``NodeBatch``, each with a subset plan,
plan.make_subset_plan).  A group larger than one batch may hold (max_batch_nodes: 56 nodes
at 2048^2) is split into several batches the same way (C5's 64 nodes on one GPU: 56 + 8).  With one batch -- every BASELINE
config at its GPU count -- the batch IS the rank:
its ``x_ext`` is exchanged in place and nothing else runs.  With several, an edge between
two groups is stored by both and updated bitwise identically at both (the single-y /
two-dual edge math is elementwise and deterministic), and each group's halo rows (other
groups' nodes, remote nodes) are filled from one rank-level image table after the
inter-rank exchange: local rows in, ``HaloExchange.run``, halo rows out -- device copies
of the same bytes, so the run is bitwise the one a single batch would do if the
operators were equal.
"""
from __future__ import annotations

import os
import warnings

import torch

from .exchange import HaloExchange, assemble_stats_device, assemble_stats_parts, gather_images_parts
import torch.distributed as dist

from .plan import STORED_Z_HBM_FRACTION, ShardPlan, make_plan, make_subset_plan, z_is_stored
from .solver import NodeBatch


def operator_key(A):
    """Nodes with equal keys share one batch (one projector context)."""
    return (A.geom, A.dtype, A.device)


# smallest batch a concurrent split makes: a full node-interleave vector (8 float32 / 4 float64
# nodes; admm_tomo.hip vb_for) -- narrower batches pay the per-tap address VALU per fewer nodes
SPLIT_MIN = {"float32": 8, "float64": 4}


def max_batch_nodes(geom) -> int:
    """Most nodes one device batch may hold: the library addresses a batch's node-interleaved
    sample buffers with 32-bit offsets (admm_batch_bind: V x max(n, m) x 8 bytes < 2^31), so
    at 2048^2 (n = 4.2 M) that is 63 nodes, rounded down to whole 8-node chunks (the widest
    interleave): 56."""
    cap = ((1 << 31) - 1) // (8 * max(geom.n, geom.m))
    return cap - cap % 8 if cap >= 8 else max(1, cap)


def rank_batches(A_list, plan: ShardPlan, streams: int = 1):
    """The device batches of one rank: [(batch key, its global nodes)] in batch order.  Nodes
    are grouped by operator key; a group larger than one batch may hold is split into
    consecutive cap-sized chunks -- not near-equal: every edge between two batches is stored
    (and updated) by both, and for a dense graph the cross edges |A| x |B| are fewest for the
    most unequal split (C5 on one GPU as 56 + 8 stores 2464 edges, as 32 + 32 it would store
    3040: +36 GB of float64 edge state); at 2048^2 an 8-node batch is two 4-node chunks of 1816
    forward blocks each, so the small batch does not idle the GPU.  ``streams`` > 1: every group
    of at least 2 x SPLIT_MIN nodes is further split into up to that many near-equal
    consecutive parts of >= SPLIT_MIN nodes (RankGroups' concurrent batches)."""
    keys, members = [], {}
    for g in plan.local_nodes:
        k = operator_key(A_list[g])
        if k not in members:
            keys.append(k)
            members[k] = []
        members[k].append(g)
    split = []
    for k in keys:
        cap = max_batch_nodes(k[0])
        nodes = members.pop(k)
        for c0 in range(0, len(nodes), cap):
            split.append((k, c0))
            members[(k, c0)] = nodes[c0:c0 + cap]
    keys = split
    if streams > 1:
        split = []
        for k in keys:
            nodes = members.pop(k)
            parts = max(1, min(streams, len(nodes) // SPLIT_MIN[k[0][1]]))
            c0 = 0
            for q in range(parts):
                sz = len(nodes) // parts + (1 if q < len(nodes) % parts else 0)
                split.append((k[0], (k[1], q)))  # (operator key, batch tag)
                members[(k[0], (k[1], q))] = nodes[c0:c0 + sz]
                c0 += sz
        keys = split
    return [(k, members[k]) for k in keys]


def stored_edges_per_rank(A_list, G, V_total: int, world: int, streams: int = 1) -> list[int]:
    """Stored edge slots of every rank of a ``world``-rank run, summed over each rank's device
    batches (rank_batches) -- what the stored-z rule (plan.z_is_stored) weighs."""
    out = []
    for r in range(world):
        pr = make_plan(G, V_total, world, r)
        if not pr.local_nodes:
            out.append(0)
            continue
        bs = rank_batches(A_list, pr, streams)
        if len(bs) == 1:
            out.append(len(pr.stored_edges))
        else:
            out.append(sum(len(make_subset_plan(G, V_total, nodes, world, r, pr.ranges, pr.edges).stored_edges)
                           for _, nodes in bs))
    return out


def min_over_ranks(value: int, world: int, group=None, device=None) -> int:
    """``value`` reduced to its minimum over the ranks of a distributed run (one all-reduce;
    gloo reduces a host tensor, RCCL a tensor on ``device``); the value itself otherwise."""
    if world > 1 and dist.is_available() and dist.is_initialized():
        gloo = dist.get_backend(group) == "gloo"
        t = torch.tensor([int(value)], dtype=torch.int64,
                         device="cpu" if gloo or device is None else torch.device("cuda", device))
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
        return int(t.item())
    return int(value)


def run_hbm_bytes(device, world: int, group=None, collective: bool = True) -> int:
    """HBM of the run's devices: this device's total memory, the minimum over ranks when the run
    is distributed (one all-reduce at setup), so a rule weighed against it is identical on
    every rank even if the devices differ."""
    hbm = int(torch.cuda.get_device_properties(device).total_memory)
    return min_over_ranks(hbm, world, group, device) if collective else hbm


class RankGroups:
    def __init__(self, A_list, G, V_total: int, world: int, rank: int, sinograms, Qij_diag_fn,
                 rho, lam, mu, tv_iters, cg_iters, tv_kind, phantom, fusion="midpoint", Wi_list=None,
                 keep_x=False, group=None, halo=True, streams=1, derive_z=None):
        """``halo=False``: no inter-rank exchange (bench.py's per-rank proxy: one rank's share
        of a ``world``-rank run on one GPU, its halo rows held fixed).  ``streams`` > 1: every
        operator group of at least 2 x SPLIT_MIN nodes is split into up to that many near-equal
        batches whose x-updates (and edge updates) run concurrently on their own HIP streams,
        so one batch's kernels fill the other's dependent-launch gaps and kernel tails; each
        batch keeps a full node-interleave width (SPLIT_MIN nodes), and the run is bitwise the
        one-batch run (the batch split never changes a node's arithmetic).
        ``derive_z`` None: the run's one edge-state rule (plan.z_is_stored over every rank's
        stored edges) unless ADMM_EDGE_STATE=stored|derived forces it; True / False force
        derived / stored z."""
        self.plan: ShardPlan = make_plan(G, V_total, world, rank)
        if not self.plan.local_nodes:
            raise ValueError(f"rank {rank} owns no graph nodes ({V_total} nodes over {world} ranks)")
        self.world = world
        self.group = group
        dev0 = A_list[self.plan.local_nodes[0]].device
        n0 = A_list[self.plan.local_nodes[0]].geom.n
        hbm = run_hbm_bytes(dev0, world, group, collective=halo)
        if streams > 1:
            # a stream split stores every cross-batch edge twice (y, and z when stored): the
            # split is dropped -- on every rank alike, from the busiest rank's extra slots -- when
            # that extra edge state would exceed the stored-z rule's HBM fraction
            extra = max(a - b for a, b in zip(stored_edges_per_rank(A_list, G, V_total, world, streams),
                                              stored_edges_per_rank(A_list, G, V_total, world, 1)))
            if extra * n0 * 16 > STORED_Z_HBM_FRACTION * hbm:
                warnings.warn(f"streams={streams} would store {extra} more edge slots on the busiest rank "
                              f"({extra * n0 * 16 / 2**30:.1f} GiB of float64 edge state): running one batch "
                              f"stream", RuntimeWarning)
                streams = 1
        self.streams_requested = streams
        bs = rank_batches(A_list, self.plan, streams)
        keys = [k for k, _ in bs]
        members = dict(bs)
        self.fusion = fusion
        forced = os.environ.get("ADMM_EDGE_STATE", "")
        if derive_z is None and forced in ("stored", "derived"):
            derive_z = forced == "derived"
        if derive_z is None and fusion == "midpoint":
            derive_z = not z_is_stored(stored_edges_per_rank(A_list, G, V_total, world, streams), n0, hbm, fusion)
        self.derive_z = bool(derive_z) if derive_z is not None else False
        devices = {k[0][2] for k in keys}
        if len(devices) > 1:
            raise ValueError("a rank's operators must all live on one device (got "
                             f"{sorted(devices)}): one process per GPU")
        if len(keys) == 1:
            plans = [self.plan]
        else:
            plans = [make_subset_plan(G, V_total, members[k], world, rank, self.plan.ranges, self.plan.edges)
                     for k in keys]
        self.batches = []
        for k, gp in zip(keys, plans):
            geom, dtype, device = k[0]
            self.batches.append(NodeBatch(geom, dtype, gp, sinograms, Qij_diag_fn, rho, lam, mu, tv_iters,
                                          cg_iters, tv_kind, phantom, device, fusion=fusion, Wi_list=Wi_list,
                                          keep_x=keep_x, derive_z=self.derive_z))
        self.device = self.batches[0].dev
        if len(self.batches) == 1:
            self.x_rank = self.batches[0].x_ext
            self.moves = []
        else:
            n = self.batches[0].x_ext.shape[1]
            self.x_rank = torch.zeros((self.plan.n_xext, n), dtype=torch.float64, device=self.device)
            row = self.plan.xrow
            lt = lambda v: torch.tensor(v, dtype=torch.long, device=self.device)  # noqa: E731
            # (batch, its local rows' slots in x_rank, x_rank slots of its halo rows)
            self.moves = [(nb, lt([row[g] for g in nb.plan.local_nodes]), lt([row[g] for g in nb.plan.halo_nodes]))
                          for nb in self.batches]
        self.halo = HaloExchange(self.plan, self.x_rank, group) if halo else None
        # one stream per batch when several run concurrently (streams > 1)
        self.streams = ([torch.cuda.Stream(device=self.device) for _ in self.batches]
                        if streams > 1 and len(self.batches) > 1 else None)

    def _concurrent(self, fn) -> None:
        """fn(nb) for every batch: in order on the current stream, or (streams > 1) each on its
        own stream, forked from and joined back into the current one."""
        if self.streams is None:
            for nb in self.batches:
                fn(nb)
            return
        cur = torch.cuda.current_stream(self.device)
        fork = cur.record_event()
        for nb, s in zip(self.batches, self.streams):
            s.wait_event(fork)
            with torch.cuda.stream(s):
                fn(nb)
        for s in self.streams:
            cur.wait_stream(s)

    @property
    def single(self) -> bool:
        return len(self.batches) == 1

    @property
    def V(self) -> int:
        return self.plan.V

    def node_update(self, rounds: int | None = None) -> None:
        self._concurrent(lambda nb: nb.node_update(rounds))

    def exchange(self) -> None:
        """Every batch's halo rows <- the current images of their nodes (other batches of
        this rank, other ranks)."""
        for nb, loc, _ in self.moves:
            self.x_rank.index_copy_(0, loc, nb.x_local)
        if self.halo is not None:
            self.halo.run()
        for nb, _, hal in self.moves:
            if hal.numel():
                torch.index_select(self.x_rank, 0, hal, out=nb.x_ext[nb.V:])

    def consensus(self) -> None:
        self._concurrent(lambda nb: nb.consensus())

    @property
    def overlaps_exchange(self) -> bool:
        """exchange_consensus can run the rank-internal edge updates under the halo exchange:
        one batch, stored z, midpoint fusion, an inter-rank exchange, and internal edges."""
        if self.halo is None or not self.halo.active or not self.single:
            return False
        nb = self.batches[0]
        return nb.z is not None and nb.fusion == "midpoint" and nb.plan.n_internal > 0

    def exchange_consensus(self) -> None:
        """``exchange()`` then ``consensus()``, with the edges whose endpoints are both local
        (stored slots [0, n_internal), x_ext rows < V) updated while the halo images are in
        flight: the exchange is issued asynchronously (RCCL on its own stream), those edges run
        on the current stream, then the halo rows land and the remaining edges run.  The same
        per-edge kernels and statistics as the serial order, bitwise."""
        if not self.overlaps_exchange or os.environ.get("ADMM_EXCHANGE_OVERLAP", "1") == "0":
            self.exchange()
            self.consensus()
            return
        nb = self.batches[0]
        h = self.halo.start()
        nb.consensus_range(0, nb.plan.n_internal, nb.V)
        self.halo.finish(h)
        nb.consensus_range(nb.plan.n_internal, len(nb.plan.stored_edges), nb.plan.n_xext)

    def stats(self, extra=None):
        """Global node / edge statistics; ``extra`` (rank-local [V, k] numpy, rows in
        plan.local_nodes order) is appended to the node statistics."""
        parts = []
        for nb in self.batches:
            ns = nb.node_stats
            if extra is not None:
                rows = [self.plan.local_nodes.index(g) for g in nb.plan.local_nodes]
                ex = torch.as_tensor(extra[rows], dtype=torch.float64, device=ns.device)
                ns = torch.cat([ns, ex], dim=1)
            parts.append((nb.plan, ns, nb.edge_stats[: len(nb.plan.stored_edges)]))
        return assemble_stats_parts(self.plan.V_total, len(self.plan.edges), self.world, parts, self.group)

    def stats_device(self) -> torch.Tensor:
        """The global statistics table on the device (exchange.assemble_stats_device): no
        host synchronisation."""
        parts = [(nb.plan, nb.node_stats, nb.edge_stats[: len(nb.plan.stored_edges)]) for nb in self.batches]
        return assemble_stats_device(self.plan.V_total, len(self.plan.edges), self.world, parts, self.group)

    def local_images(self):
        """[(global node, image row tensor)] of this rank's nodes, ascending."""
        out = []
        for nb in self.batches:
            out.extend((g, nb.x_local[r]) for r, g in enumerate(nb.plan.local_nodes))
        return sorted(out, key=lambda t: t[0])

    def images(self) -> torch.Tensor:
        return gather_images_parts(self.plan.V_total, self.world,
                                   [(nb.plan, nb.x_local) for nb in self.batches], self.group)
