"""Halo exchange of node images and deterministic statistics assembly.

One process per GPU; ``torch.distributed`` with backend "nccl" is RCCL over
xGMI on ROCm ("gloo" on CPU tensors in the tests).  The only per-iteration
data exchange of the ADMM loop is x_j of remote neighbours (plan.py):

* sparse graphs (ring): grouped point-to-point send/recv of the boundary
  images straight into the contiguous halo rows of ``x_ext``;
* dense / Erdos-Renyi graphs: one all-gather of every rank's images.

Per-node and per-edge statistics are summed with one all-reduce of a
zero-padded vector in which exactly one rank writes each entry, so the result
is bitwise what a single GPU computes (x + 0 = x).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .plan import ShardPlan


class HaloExchange:
    def __init__(self, plan: ShardPlan, x_ext: torch.Tensor, group=None):
        self.plan = plan
        self.x = x_ext
        self.group = group
        self.active = plan.world > 1
        if not self.active:
            return
        dev = x_ext.device
        # gloo moves host tensors only: device images are staged through host copies
        # (tests and 1-GPU rehearsals; RCCL reads and writes HBM directly)
        self.stage = x_ext.is_cuda and dist.get_backend(group) == "gloo"
        self.mode = "allgather" if plan.use_allgather() else "p2p"
        V = plan.V
        if self.mode == "allgather":
            counts = [hi - lo for lo, hi in plan.ranges]
            self.vmax = max(counts)
            n = x_ext.shape[1]
            self.sendbuf = torch.zeros((self.vmax, n), dtype=x_ext.dtype, device=dev)
            self.full = torch.zeros((plan.world * self.vmax, n), dtype=x_ext.dtype, device=dev)
            idx = []
            for g in plan.halo_nodes:
                r = next(r for r, (lo, hi) in enumerate(plan.ranges) if lo <= g < hi)
                idx.append(r * self.vmax + (g - plan.ranges[r][0]))
            self.halo_idx = torch.tensor(idx, dtype=torch.long, device=dev)
        else:
            self.sends = []
            for peer, nodes in sorted(plan.send.items()):
                if nodes:
                    rows = torch.tensor([plan.xrow[g] for g in nodes], dtype=torch.long, device=dev)
                    buf = torch.empty((len(nodes), x_ext.shape[1]), dtype=x_ext.dtype, device=dev)
                    self.sends.append((peer, rows, buf))
            self.recvs = []
            for peer, nodes in sorted(plan.recv.items()):
                if nodes:
                    r0 = plan.xrow[nodes[0]]
                    assert [plan.xrow[g] for g in nodes] == list(range(r0, r0 + len(nodes)))
                    self.recvs.append((peer, r0, len(nodes)))
        self.V = V

    def run(self) -> None:
        self.finish(self.start())

    def start(self):
        """Issue the exchange (asynchronous collectives: RCCL runs them on its own stream after
        the work already enqueued on the current one); ``finish`` lands the halo rows.  Work
        enqueued on the current stream between the two -- kernels that read only the local rows
        -- runs while the images are in flight."""
        if not self.active:
            return None
        p = self.plan
        if self.mode == "allgather":
            self.sendbuf[: self.V].copy_(self.x[: self.V])
            if self.stage:
                full = self.full.cpu()
                return ("ag", dist.all_gather_into_tensor(full, self.sendbuf.cpu(), group=self.group,
                                                          async_op=True), full)
            return ("ag", dist.all_gather_into_tensor(self.full, self.sendbuf, group=self.group, async_op=True),
                    None)
        ops, landing = [], []
        for peer, rows, buf in self.sends:
            torch.index_select(self.x, 0, rows, out=buf)
            ops.append(dist.P2POp(dist.isend, buf.cpu() if self.stage else buf, peer, group=self.group))
        for peer, r0, cnt in self.recvs:
            dst = self.x[r0:r0 + cnt]
            if self.stage:
                host = torch.empty(dst.shape, dtype=dst.dtype)
                landing.append((dst, host))
                dst = host
            ops.append(dist.P2POp(dist.irecv, dst, peer, group=self.group))
        return ("p2p", dist.batch_isend_irecv(ops) if ops else [], landing)

    def finish(self, h) -> None:
        if h is None:
            return
        kind, work, extra = h
        if kind == "ag":
            work.wait()
            if extra is not None:
                self.full.copy_(extra)
            if len(self.plan.halo_nodes):
                self.x[self.V:].copy_(self.full.index_select(0, self.halo_idx))
            return
        for req in work:
            req.wait()
        for dst, host in extra:
            dst.copy_(host)


def _all_reduce_sum(t: torch.Tensor, group=None) -> torch.Tensor:
    if t.is_cuda and dist.get_backend(group) == "gloo":
        host = t.cpu()
        dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
        t.copy_(host)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def assemble_stats(plan: ShardPlan, node_stats: torch.Tensor, edge_stats: torch.Tensor, group=None):
    """Global (V_total, ns) node and (E_total, es) edge statistics as float64 CPU tensors."""
    return assemble_stats_parts(plan.V_total, len(plan.edges), plan.world,
                                [(plan, node_stats, edge_stats)], group)


def assemble_stats_parts(V_total: int, E: int, world: int, parts, group=None):
    """Statistics of several batches (``parts`` = [(plan, node_stats, edge_stats)], one per
    node batch of this rank) as global (V_total, ns) / (E, es) float64 CPU tensors.  Every
    entry has exactly one writer -- the batch holding the node, the batch owning the edge
    (lower endpoint) -- into a zero table, so the values are the writers' bits (x + 0 = x)
    however the nodes are split over batches and ranks."""
    plan0, ns0, es0 = parts[0]
    ns = ns0.shape[1]
    es = es0.shape[1] if es0 is not None else 3
    if world == 1 and len(parts) == 1:
        nodes = ns0.detach().to("cpu")
        edges = torch.zeros((E, es), dtype=torch.float64)
        if E and plan0.stored_edges:
            edges[torch.tensor(plan0.stored_edges, dtype=torch.long)] = es0.detach().to("cpu")
        return nodes, edges
    return split_stats(assemble_stats_device(V_total, E, world, parts, group).to("cpu"), V_total, ns, E, es)


def assemble_stats_device(V_total: int, E: int, world: int, parts, group=None) -> torch.Tensor:
    """The global statistics table of ``assemble_stats_parts`` left on the device, flat
    ([V_total x ns | E x es] float64): stream-ordered, no host synchronisation (an RCCL
    all-reduce at world > 1), for loops that read it back later (run_admm's pipelined mode,
    bench.py).  ``split_stats`` cuts a host copy into the (nodes, edges) pair."""
    plan0, ns0, es0 = parts[0]
    ns = ns0.shape[1]
    es = es0.shape[1] if es0 is not None else 3
    dev = ns0.device
    if world == 1 and len(parts) == 1 and plan0.stored_edges == list(range(E)):
        # one batch holding every node and every edge in G.edges() order: the table is its
        # two statistics arrays back to back (one copy kernel)
        return torch.cat([ns0.reshape(-1), es0[:E].reshape(-1)]) if E else ns0.reshape(-1).clone()
    buf = torch.zeros(V_total * ns + E * es, dtype=torch.float64, device=dev)
    nv = buf[: V_total * ns].view(V_total, ns)
    ev = buf[V_total * ns:].view(E, es)
    for plan, node_stats, edge_stats in parts:
        if plan.V:
            nv.index_copy_(0, _index(plan, "local", dev), node_stats)
        owned = _index(plan, "owned_slots", dev)
        if owned.numel():
            ev.index_copy_(0, _index(plan, "owned_gids", dev), edge_stats.index_select(0, owned))
    if world > 1:
        _all_reduce_sum(buf, group)
    return buf


def split_stats(flat: torch.Tensor, V_total: int, ns: int, E: int, es: int):
    return flat[: V_total * ns].view(V_total, ns), flat[V_total * ns:].view(E, es)


def _index(plan: ShardPlan, what: str, dev) -> torch.Tensor:
    """Device index tensors of a plan, built once (the statistics are assembled every
    iteration)."""
    cache = plan.__dict__.setdefault("_idx_cache", {})
    key = (what, str(dev))
    t = cache.get(key)
    if t is None:
        owned = [k for k, o in enumerate(plan.owned_edge) if o]
        vals = {"local": plan.local_nodes, "owned_slots": owned,
                "owned_gids": [plan.stored_edges[k] for k in owned]}[what]
        t = torch.tensor(vals, dtype=torch.long, device=dev)
        cache[key] = t
    return t


def gather_images(plan: ShardPlan, x_local: torch.Tensor, group=None) -> torch.Tensor:
    """(V_total, n) float64 images of every node on every rank (end of the loop)."""
    return gather_images_parts(plan.V_total, plan.world, [(plan, x_local)], group)


def gather_images_parts(V_total: int, world: int, parts, group=None) -> torch.Tensor:
    """``parts`` = [(plan, x_local)] of this rank's batches -> (V_total, n) images (one
    writer per row, summed over ranks)."""
    plan0, x0 = parts[0]
    if world == 1 and len(parts) == 1:
        return x0
    n = x0.shape[1]
    buf = torch.zeros((V_total, n), dtype=x0.dtype, device=x0.device)
    for plan, x_local in parts:
        if plan.V:
            buf.index_copy_(0, torch.tensor(plan.local_nodes, dtype=torch.long, device=x0.device), x_local)
    return _all_reduce_sum(buf, group) if world > 1 else buf


def _row_digest(rows: torch.Tensor) -> torch.Tensor:
    """Per-row int64 digest of the rows' bytes (position-weighted, wrapping int64 sums):
    equal bytes give equal digests, any changed element changes it almost surely."""
    v = rows.contiguous().view(torch.int64) if rows.dtype == torch.float64 else \
        rows.contiguous().view(torch.int32).to(torch.int64)
    w = torch.arange(v.shape[1], device=v.device, dtype=torch.int64) * 2 + 1
    return (v * w).sum(dim=1)


def verify_halo(plan: ShardPlan, x_ext: torch.Tensor, group=None) -> dict:
    """Check that every halo row of ``x_ext`` holds, byte for byte, the owner rank's
    current image of that node (what ``HaloExchange.run`` must deliver, by p2p or
    all-gather).  Each rank contributes the digests of its own nodes to one table
    (one all-reduce; exactly one rank writes each entry) and compares its halo rows.
    Returns {"halo_rows", "mismatched_rows"} summed over ranks."""
    if plan.world == 1:
        return {"halo_rows": 0, "mismatched_rows": 0}
    dev = x_ext.device
    tbl = torch.zeros(plan.V_total, dtype=torch.int64, device=dev)
    lo = plan.local_nodes[0] if plan.local_nodes else 0
    if plan.V:
        tbl[lo:lo + plan.V] = _row_digest(x_ext[: plan.V])
    _all_reduce_sum(tbl, group)
    bad = 0
    if plan.halo_nodes:
        rows = torch.tensor([plan.xrow[g] for g in plan.halo_nodes], dtype=torch.long, device=dev)
        want = tbl[torch.tensor(plan.halo_nodes, dtype=torch.long, device=dev)]
        bad = int((_row_digest(x_ext.index_select(0, rows)) != want).sum().item())
    counts = torch.tensor([len(plan.halo_nodes), bad], dtype=torch.int64, device=dev)
    _all_reduce_sum(counts, group)
    return {"halo_rows": int(counts[0].item()), "mismatched_rows": int(counts[1].item())}

