"""Graph-node sharding plan: which nodes, edges and halo images live on a rank.

Pure host logic (no GPU), exercised by the world-size-2 gloo tests.

* Nodes are split into contiguous blocks, one per rank; within a rank,
  nodes whose operators differ (unequal angle counts, different matrices) form separate
  batches, each with a subset plan (``make_subset_plan``; admm_hip/groups.py).
* Edges are the reference's ``G.edges()`` in order, canonicalised to
  (min, max) (block_6_admm_loop_ver2.py:39-43,211-212).  A rank stores every
  edge incident to one of its nodes; an edge whose endpoints live on two ranks
  is stored (and updated, bitwise identically) on both.  Its statistics are
  reported by the owner of the lower endpoint.
* The only data a rank needs from others is x_j of its halo nodes (remote
  neighbours): with the single-y edge form z and y are computed redundantly
  at both ends, so no second exchange is needed.
* Incident edge-ends of a node are listed in ``G.neighbors(i)`` order so the
  neighbour sums c_i = sum_j q_ij v_ij add in the reference's order
  (block_6_admm_loop_ver2.py:87).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np


def node_ranges(V: int, world: int) -> list[tuple[int, int]]:
    """Contiguous near-equal blocks [lo, hi) of graph nodes per rank."""
    bounds = np.linspace(0, V, world + 1)
    cuts = [int(round(b)) for b in bounds]
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def owner_of(ranges: list[tuple[int, int]], node: int) -> int:
    for r, (lo, hi) in enumerate(ranges):
        if lo <= node < hi:
            return r
    raise KeyError(node)


@dataclass
class ShardPlan:
    V_total: int
    world: int
    rank: int
    edges: list  # global canonical edges (a, b), a < b, in G.edges() order
    ranges: list
    local_nodes: list = field(default_factory=list)
    halo_nodes: list = field(default_factory=list)
    xrow: dict = field(default_factory=dict)        # global node -> x_ext row
    stored_edges: list = field(default_factory=list)  # global edge ids stored here
    edge_a_row: list = field(default_factory=list)
    edge_b_row: list = field(default_factory=list)
    owned_edge: list = field(default_factory=list)  # bool per stored edge
    n_internal: int = 0  # stored slots [0, n_internal): both endpoints local (x_ext rows < V)
    inc_off: list = field(default_factory=list)
    inc_edge: list = field(default_factory=list)    # stored-edge slot
    inc_nbr: list = field(default_factory=list)     # neighbour global id (for Qij_diag_fn)
    inc_sign: list = field(default_factory=list)
    send: dict = field(default_factory=dict)        # peer -> sorted local nodes it needs
    recv: dict = field(default_factory=dict)        # peer -> sorted halo nodes it sends

    @property
    def V(self) -> int:
        return len(self.local_nodes)

    @property
    def n_xext(self) -> int:
        return len(self.local_nodes) + len(self.halo_nodes)

    def use_allgather(self) -> bool:
        """All-gather only when it moves no more bytes to the busiest rank than p2p would:
        an all-gather lands (world - 1) x vmax images on every rank, the grouped p2p exactly
        a rank's halo rows, so p2p wins unless some rank needs (nearly) every remote image --
        complete graphs (C5).  C4's 32-node ER graph on 8 ranks: at most 20 halo rows against
        28 all-gathered images per rank.  (Round 4's rule all-gathered whenever a rank needed
        more than half its remote images.)

        The exchange is a collective, so the choice is made from the whole graph and node
        partition -- the same on every rank (a rank-local choice let C4's 32-node ER graph
        on 8 ranks put one rank in p2p mode while the others all-gathered: a deadlock)."""
        if self.world == 1:
            return False
        cached = self.__dict__.get("_allgather")
        if cached is None:
            owner = np.empty(self.V_total, dtype=np.int64)
            for r, (lo, hi) in enumerate(self.ranges):
                owner[lo:hi] = r
            halo = [set() for _ in range(self.world)]
            for a, b in self.edges:
                ra, rb = int(owner[a]), int(owner[b])
                if ra != rb:
                    halo[ra].add(b)
                    halo[rb].add(a)
            vmax = max(hi - lo for lo, hi in self.ranges)
            busiest = max(len(h) for h in halo)
            cached = busiest > 0 and busiest >= (self.world - 1) * vmax
            self.__dict__["_allgather"] = cached
        return cached


def canonical_edges(G, V_total: int) -> list:
    """``G.edges()`` as (min, max) pairs in order, validated (block_6_admm_loop_ver2.py:39-43)."""
    edges = [(min(i, j), max(i, j)) for i, j in G.edges()]
    if len(set(edges)) != len(edges):
        raise ValueError("graph has duplicate edges")
    for a, b in edges:
        if a == b:
            raise ValueError("self loops are not supported")
        if not (0 <= a < V_total and 0 <= b < V_total):
            raise ValueError("edge endpoint out of range")
    return edges


def make_subset_plan(G, V_total: int, nodes, world: int = 1, rank: int = 0, ranges=None,
                     edges=None) -> ShardPlan:
    """Plan of an arbitrary set of graph nodes held by one batch: its local rows (``nodes``
    in ascending order), the halo rows of every neighbour outside the set, the stored edges
    (every edge incident to the set) and the incidence lists.  An edge is owned (its
    statistics reported) by the batch holding its lower endpoint."""
    if edges is None:
        edges = canonical_edges(G, V_total)
    P = ShardPlan(V_total=V_total, world=world, rank=rank, edges=edges,
                  ranges=ranges if ranges is not None else [(0, V_total)])
    P.local_nodes = sorted(int(g) for g in nodes)
    local = set(P.local_nodes)
    halo = set()
    for a, b in edges:
        if a in local and b not in local:
            halo.add(b)
        if b in local and a not in local:
            halo.add(a)
    P.halo_nodes = sorted(halo)
    for r, g in enumerate(P.local_nodes + P.halo_nodes):
        P.xrow[g] = r
    # stored edge slots: the set's internal edges (both endpoints local, x_ext rows < V) first,
    # then the edges to halo nodes, each in G.edges() order -- so the internal ones can be
    # updated while the halo exchange is still writing rows >= V (admm_consensus_range); the
    # per-edge arithmetic does not depend on the slot
    internal = [ge for ge, (a, b) in enumerate(edges) if a in local and b in local]
    boundary = [ge for ge, (a, b) in enumerate(edges) if (a in local) != (b in local)]
    P.n_internal = len(internal)
    eidx = {}
    for ge in internal + boundary:
        a, b = edges[ge]
        eidx[ge] = len(P.stored_edges)
        P.stored_edges.append(ge)
        P.edge_a_row.append(P.xrow[a])
        P.edge_b_row.append(P.xrow[b])
        P.owned_edge.append(a in local)
    edge_of = {e: ge for ge, e in enumerate(edges)}
    P.inc_off = [0]
    for g in P.local_nodes:
        for j in G.neighbors(g):
            e = (min(g, j), max(g, j))
            P.inc_edge.append(eidx[edge_of[e]])
            P.inc_nbr.append(int(j))
            P.inc_sign.append(1 if g == e[0] else -1)
        P.inc_off.append(len(P.inc_edge))
    return P


def make_plan(G, V_total: int, world: int = 1, rank: int = 0) -> ShardPlan:
    """Plan of rank ``rank``: the contiguous node block node_ranges(V_total, world)[rank],
    plus which boundary images it sends to / receives from every peer."""
    edges = canonical_edges(G, V_total)
    ranges = node_ranges(V_total, world)
    lo, hi = ranges[rank]
    P = make_subset_plan(G, V_total, range(lo, hi), world, rank, ranges, edges)
    local = set(P.local_nodes)
    for peer in range(world):
        if peer == rank:
            continue
        plo, phi = ranges[peer]
        P.recv[peer] = [g for g in P.halo_nodes if plo <= g < phi]
        need = set()
        for a, b in edges:
            if a in local and plo <= b < phi:
                need.add(a)
            if b in local and plo <= a < phi:
                need.add(b)
        P.send[peer] = sorted(need)
    return P


# --------------------------------------------------------------------------------------
# Edge-state rule: stored z or z derived from x_prev (ABI 7)
# --------------------------------------------------------------------------------------
# Fraction of a GPU's HBM the float64 edge state of its busiest rank may take with z stored
# (y and z: two rows of n pixels per stored edge slot).  Stored z is the faster edge state
# wherever it fits (C4 rank 3 of 8: 8.67 vs 8.98 ms per step; C5 rank 0 of 8: 143 vs 154 ms;
# profiles/r4_shares_derived_vs_stored_z.txt): the gather / DIAG / consensus read one z row per
# incidence instead of the two endpoint rows of x_prev.  Derived z halves the edge state, so it
# is kept for graphs whose stored state would not fit.  Every BASELINE config fits at every GPU
# count; the fullest is C5 on one GPU: 2464 stored edges x 2 x 33.5 MB = 165 GB against
# 0.6 x 288 GB = 173 GB, leaving ~70 GB for the node state and scratch (~55 GB).
STORED_Z_HBM_FRACTION = 0.6


def stored_edge_state_bytes(stored_edges_per_rank, n: int) -> int:
    """Bytes of the float64 edge state (y and z, one row of n pixels each per stored edge slot)
    on the busiest rank; ``stored_edges_per_rank``: every rank's stored edge slots, summed over
    its device batches (an edge between two batches of one rank is stored by both)."""
    return max(stored_edges_per_rank) * n * 8 * 2


def z_is_stored(stored_edges_per_rank, n: int, hbm_bytes: int, fusion: str = "midpoint",
                fraction: float = STORED_Z_HBM_FRACTION) -> bool:
    """The one edge-state rule of a run: stored z iff the busiest rank's y and z rows fit in
    ``fraction`` of ``hbm_bytes`` (weighted fusion always stores z).  A function of the whole
    run -- every rank's stored edges, the image size and the devices' HBM -- so every rank gets
    the same answer: derived and stored z differ in the last bits, and an edge stored on two
    ranks (or two batches) must be updated bitwise identically at both ends."""
    if fusion != "midpoint":
        return True
    return stored_edge_state_bytes(stored_edges_per_rank, n) <= fraction * hbm_bytes
