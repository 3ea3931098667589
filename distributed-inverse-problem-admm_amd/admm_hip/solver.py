"""Device-resident node batch: the per-GPU state of the decentralized ADMM hot path.

Holds, in HBM, everything one GPU needs for its graph nodes (layout: DESIGN.md
"Data layout in HBM") and drives the C-ABI entry points:

* ``node_update()``  -- x-update of every local node (admm_node_update; replaces
  block_6_admm_loop_ver2.py:81-197: neighbour gather, CVXPY/SCS solve, g check);
* ``consensus()``    -- z / y / residual partials of every stored edge
  (admm_consensus; replaces block_6_admm_loop_ver2.py:210-253).

Both are stream-ordered on the current torch stream and replay hipGraphs
recorded at bind time.  ``keep_x=True`` promises that nothing but ``node_update``
writes the local rows of ``x_ext``; each update then starts from the previous
update's A^T(Ax - b) instead of projecting x again (ADMM_BATCH_KEEP_X).
"""
from __future__ import annotations

import ctypes as C
import hashlib

import numpy as np
import torch

from . import _lib
from .geometry import ParallelBeamGeometry, RayTransform, current_stream_handle, _Ctx
from .plan import ShardPlan, z_is_stored


def _as_f64_tensor(v, n: int, dev) -> torch.Tensor:
    t = torch.as_tensor(v) if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v))
    t = t.reshape(-1)
    if t.numel() != n:
        raise ValueError(f"vector has {t.numel()} entries, expected {n}")
    return t.to(device=dev, dtype=torch.float64)


def _vec_key(t: torch.Tensor):
    h = hashlib.blake2b(t.detach().to("cpu").numpy().tobytes(), digest_size=16).hexdigest()
    return ("hash", h)


class NodeBatch:
    def __init__(self, geom: ParallelBeamGeometry, dtype: str, plan: ShardPlan, sinograms,
                 Qij_diag_fn, rho: float, lam: float, mu: float, tv_iters: int = 10,
                 cg_iters: int = 5, tv_kind: str = "iso", phantom=None, device: int = 0,
                 fusion: str = "midpoint", Wi_list=None, keep_x: bool = False, derive_z: bool | None = None):
        """``derive_z``: z_ij is not stored but derived from the endpoint images of the last
        consensus (``x_prev``, one row per x_ext row; ABI 7; midpoint fusion only).  None: the
        edge-state rule (plan.z_is_stored) on this batch alone -- stored z, the faster form,
        unless its rows would exceed the rule's share of HBM; RankGroups passes the run's one
        global decision instead.  block_5's drop-in, which injects arbitrary targets v_ij through
        z, keeps it stored (``derive_z=False``)."""
        self.lib = _lib.load()
        self.geom = geom
        self.plan = plan
        self.dtype = dtype
        self.device = device
        dev = torch.device("cuda", device)
        self.dev = dev
        n, m = geom.n, geom.m
        V = plan.V
        if V < 1:
            raise ValueError("rank owns no graph nodes")
        sdt = torch.float64 if dtype == "float64" else torch.float32
        self.ctx = _Ctx(geom, dtype, device, max_images=max(1, V))
        self.x_ext = torch.zeros((plan.n_xext, n), dtype=torch.float64, device=dev)
        self.d = torch.zeros((V, 2, n), dtype=torch.float64, device=dev)
        self.e = torch.zeros((V, 2, n), dtype=torch.float64, device=dev)
        self.atb = torch.zeros((V, n), dtype=torch.float64, device=dev)
        self.b = torch.empty((V, m), dtype=sdt, device=dev)
        for k, g in enumerate(plan.local_nodes):
            s = sinograms[g]
            st = s if isinstance(s, torch.Tensor) else torch.as_tensor(np.asarray(s))
            st = st.reshape(-1)
            if st.numel() != m:
                raise ValueError(f"sinogram of node {g} has {st.numel()} entries, expected {m}")
            self.b[k].copy_(st.to(device=dev, dtype=sdt))
        self.phantom = None
        if phantom is not None:
            self.phantom = _as_f64_tensor(phantom, n, dev)
        # precision vectors q_ij, deduplicated into slots
        E = len(plan.stored_edges)
        keyfn = getattr(Qij_diag_fn, "qslot_key", None)
        slots, qvecs, inc_qslot = {}, [], []
        for k, g in enumerate(plan.local_nodes):
            for q in range(plan.inc_off[k], plan.inc_off[k + 1]):
                j = plan.inc_nbr[q]
                key = keyfn(g, j) if keyfn is not None else None
                if key is not None and key in slots:
                    inc_qslot.append(slots[key])
                    continue
                vec = _as_f64_tensor(Qij_diag_fn(g, j), n, dev)
                if key is None:
                    key = _vec_key(vec)
                if key not in slots:
                    slots[key] = len(qvecs)
                    qvecs.append(vec)
                inc_qslot.append(slots[key])
        self.q = torch.stack(qvecs) if qvecs else torch.zeros((1, n), dtype=torch.float64, device=dev)
        self.n_qslots = len(qvecs)
        self.inc_qslot_host = list(inc_qslot)
        ii = lambda a: torch.tensor(a if len(a) else [0], dtype=torch.int32, device=dev)  # noqa: E731
        self.inc_off = ii(plan.inc_off)
        self.inc_edge = ii(plan.inc_edge)
        self.inc_sign = ii(plan.inc_sign)
        self.inc_qslot = ii(inc_qslot)
        self.edge_a = ii(plan.edge_a_row)
        self.edge_b = ii(plan.edge_b_row)
        self.y = torch.zeros((max(E, 1), n), dtype=torch.float64, device=dev)
        # weighted edge fusion: both endpoint duals + W of every x_ext row
        if fusion not in ("midpoint", "weighted"):
            raise ValueError("fusion must be 'midpoint' or 'weighted'")
        if derive_z is None:
            hbm = int(torch.cuda.get_device_properties(dev).total_memory)
            derive_z = not z_is_stored([E], n, hbm, fusion)
        if derive_z and fusion != "midpoint":
            raise ValueError("derived z needs midpoint fusion")
        self.derive_z = bool(derive_z)
        # derived: x_ext at the last consensus (x = 0 before the first: z = 0); stored: z per edge
        self.z = None if self.derive_z else torch.zeros((max(E, 1), n), dtype=torch.float64, device=dev)
        self.x_prev = torch.zeros((plan.n_xext, n), dtype=torch.float64, device=dev) if self.derive_z else None
        self.fusion = fusion
        self.y_b = None
        self.w = None
        if fusion == "weighted":
            if Wi_list is None:
                raise ValueError("weighted fusion needs Wi_list")
            self.y_b = torch.zeros((max(E, 1), n), dtype=torch.float64, device=dev)
            self.w = torch.stack([_as_f64_tensor(Wi_list[g], n, dev)
                                  for g in plan.local_nodes + plan.halo_nodes])
        # D_i = sum_j q_ij  (constant across iterations; setup)
        self.dsum = torch.zeros((V, n), dtype=torch.float64, device=dev)
        for k in range(V):
            for q in range(plan.inc_off[k], plan.inc_off[k + 1]):
                self.dsum[k] += self.q[inc_qslot[q]]
        self.node_stats = torch.zeros((V, _lib.NODE_STATS), dtype=torch.float64, device=dev)
        self.edge_stats = torch.zeros((max(E, 1), _lib.EDGE_STATS), dtype=torch.float64, device=dev)
        self.params = dict(rho=float(rho), lam=float(lam), mu=float(mu), tv_iters=int(tv_iters),
                           cg_iters=int(cg_iters), tv_kind=tv_kind)
        p = lambda t: C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)  # noqa: E731
        self.cb = _lib.Batch(
            V, plan.n_xext, E, int(tv_iters), int(cg_iters),
            _lib.ADMM_TV_ANISO if tv_kind == "aniso" else _lib.ADMM_TV_ISO,
            float(rho), float(lam), float(mu),
            p(self.x_ext), p(self.d), p(self.e), p(self.atb), p(self.dsum), p(self.b), p(self.phantom),
            p(self.y), p(self.z), p(self.q), p(self.edge_a), p(self.edge_b), p(self.inc_off),
            p(self.inc_edge), p(self.inc_qslot), p(self.inc_sign), p(self.node_stats),
            p(self.edge_stats),
            _lib.ADMM_FUSE_WEIGHTED if fusion == "weighted" else _lib.ADMM_FUSE_MIDPOINT,
            _lib.ADMM_BATCH_KEEP_X if keep_x else 0,
            p(self.y_b), p(self.w), p(self.x_prev))
        torch.cuda.synchronize(dev)
        _lib.check(self.lib.admm_batch_bind(self.ctx.h, C.byref(self.cb)), "admm_batch_bind")
        _lib.check(self.lib.admm_batch_atb(self.ctx.h, p(self.atb), C.c_void_p(self._s())),
                   "admm_batch_atb")

    def set_precisions(self, qs) -> None:
        """New q_ij for a batch bound with one q slot per incidence (in incidence order): the
        slots are rewritten, D = sum_j q_ij is recomputed as at construction (same order) and the
        batch re-bound (its interleaved D samples and recorded sequences are bind-time data).
        Used by the block_5 drop-in's batch cache."""
        if len(qs) != len(self.inc_qslot_host) or sorted(self.inc_qslot_host) != list(range(len(qs))):
            raise ValueError("set_precisions needs one q slot per incidence")
        for s, q in enumerate(qs):
            self.q[self.inc_qslot_host[s]].copy_(_as_f64_tensor(q, self.geom.n, self.dev))
        self.dsum.zero_()
        for k in range(self.V):
            for s in range(self.plan.inc_off[k], self.plan.inc_off[k + 1]):
                self.dsum[k] += self.q[self.inc_qslot_host[s]]
        torch.cuda.synchronize(self.dev)
        _lib.check(self.lib.admm_batch_bind(self.ctx.h, C.byref(self.cb)), "admm_batch_bind")

    def z_of(self, k: int) -> torch.Tensor:
        """z of stored edge slot k: the stored vector, or (derived) the midpoint of its endpoint
        rows of x_prev -- the value every kernel forms."""
        if self.z is not None:
            return self.z[k]
        return (self.x_prev[self.plan.edge_a_row[k]] + self.x_prev[self.plan.edge_b_row[k]]) * 0.5

    def _s(self) -> int:
        return current_stream_handle(self.dev)

    @property
    def V(self) -> int:
        return self.plan.V

    def _info(self) -> tuple[int, bool]:
        vb, mm = C.c_int(), C.c_int()
        _lib.check(self.lib.admm_batch_info(self.ctx.h, C.byref(vb), C.byref(mm)), "admm_batch_info")
        return vb.value, bool(mm.value)

    @property
    def ctx_vb(self) -> int:
        """Node-interleave width the library chose for this batch (admm_batch_info, ABI 8):
        vb_for(V) in admm_tomo.hip, capped at 16-byte vectors in mirror mode."""
        return self._info()[0]

    @property
    def mirror(self) -> bool:
        """The bound batch's projectors run in mirror mode (admm_batch_info, ABI 8)."""
        return self._info()[1]

    @property
    def x_local(self) -> torch.Tensor:
        return self.x_ext[: self.plan.V]

    def node_update(self, rounds: int | None = None) -> None:
        """One x-update of every local node; ``rounds`` overrides the bound split-Bregman
        round count (chunked solves, admm_node_update_rounds)."""
        if rounds is None:
            _lib.check(self.lib.admm_node_update(self.ctx.h, C.c_void_p(self._s())), "admm_node_update")
        else:
            _lib.check(self.lib.admm_node_update_rounds(self.ctx.h, int(rounds), C.c_void_p(self._s())),
                       "admm_node_update_rounds")

    def node_update_masked(self, active) -> None:
        """x-update of the nodes where ``active`` (bool, length V) is set; the others keep
        their x, d, e and statistics bitwise (saved before, restored after the batched
        update).  Needs keep_x=False: a restored node's x no longer matches the kept
        A^T(Ax - b) of the reuse start."""
        act = torch.as_tensor(np.asarray(active, dtype=bool))
        if bool(act.all()):
            self.node_update()
            return
        if not bool(act.any()):
            return
        if self.cb.flags & _lib.ADMM_BATCH_KEEP_X:
            raise RuntimeError("node_update_masked needs a batch bound with keep_x=False")
        idx = torch.nonzero(~act).reshape(-1).to(self.dev)
        saved = [(t, t.index_select(0, idx)) for t in (self.x_local, self.d, self.e, self.node_stats)]
        self.node_update()
        for t, s in saved:
            t.index_copy_(0, idx, s)

    def consensus(self) -> None:
        if self.plan.stored_edges:
            _lib.check(self.lib.admm_consensus(self.ctx.h, C.c_void_p(self._s())), "admm_consensus")

    def consensus_range(self, e0: int, e1: int, rows: int) -> None:
        """Edge updates of stored slots [e0, e1) only, whose endpoints lie in x_ext rows [0, rows)
        (stored z, midpoint fusion; admm_consensus_range, ABI 9): the same per-edge results and
        statistics as ``consensus``.  The endpoint rows are checked here against ``rows`` (the
        library reads only rows below it while the halo rows may still be landing)."""
        if e1 > e0:
            top = max(max(self.plan.edge_a_row[e0:e1]), max(self.plan.edge_b_row[e0:e1]))
            if top >= rows:
                raise ValueError(f"edge slots [{e0}, {e1}) reach x_ext row {top} >= rows={rows}")
            _lib.check(self.lib.admm_consensus_range(self.ctx.h, int(e0), int(e1), int(rows), C.c_void_p(self._s())),
                       "admm_consensus_range")

    def marker(self) -> None:
        """One k_tv_grad launch (never part of an x-update or consensus): delimits the
        bench's timed steps in rocprofv3 PMC traces (scripts/traffic_summary.py)."""
        if getattr(self, "_mk", None) is None:
            self._mk = torch.empty((2, self.geom.n), dtype=torch.float64, device=self.dev)
        _lib.check(self.lib.admm_tv_grad(self.ctx.h, C.c_void_p(self.x_ext.data_ptr()),
                                         C.c_void_p(self._mk[0].data_ptr()),
                                         C.c_void_p(self._mk[1].data_ptr()), 1, C.c_void_p(self._s())),
                   "admm_tv_grad")

    def time_forward(self, reps: int = 20, in_solve: bool = False) -> float:
        """Average k_fwdg launch (ms): ``reps`` back-to-back, or ``in_solve`` -- every CG-step
        forward of one directly enqueued x-update (the batch's state advances by it)."""
        ms = C.c_double()
        _lib.check(self.lib.admm_time_forward(self.ctx.h, reps, int(in_solve), C.c_void_p(self._s()), C.byref(ms)),
                   "admm_time_forward")
        return ms.value

    def time_back(self) -> float:
        """Average in-solve back projector launch (ms; k_back / k_back_mirror in H mode): every
        CG step of one directly enqueued x-update (admm_time_back, ABI 9; the state advances)."""
        ms = C.c_double()
        _lib.check(self.lib.admm_time_back(self.ctx.h, C.c_void_p(self._s()), C.byref(ms)), "admm_time_back")
        return ms.value

    def fwd_plans(self) -> list[dict]:
        """The grouped forward projector's plans for this batch's geometry (admm_fwd_plan_info):
        per plan 0-5 its angle groups, blocks per node chunk, staged row pixels (host model)
        and whether it is the bound one; plans the geometry does not have are omitted."""
        out = []
        for pl in range(6):
            g, b, a, st = C.c_int(), C.c_int(), C.c_int(), C.c_double()
            _lib.check(self.lib.admm_fwd_plan_info(self.ctx.h, pl, C.byref(g), C.byref(b), C.byref(st),
                                                   C.byref(a)), "admm_fwd_plan_info")
            if g.value:
                out.append(dict(plan=pl, groups=g.value, blocks=b.value, staged_px=st.value,
                                active=bool(a.value)))
        return out


def make_operators(N: int, num_nodes: int, angles_total: int | None = None, dtype: str = "float32",
                   device: int | None = None, det_width_factor: float = 1.0) -> list[RayTransform]:
    """Per-node ray transforms of block_2_load_odl_data.py:16-65 (all nodes span [0, pi)),
    on ``device`` (default: the current device, see geometry.default_device)."""
    from .geometry import default_device, split_angles
    if device is None:
        device = default_device()
    if angles_total is None:
        angles_total = max(180, 3 * N)
    per = split_angles(angles_total, num_nodes)
    return [RayTransform(ParallelBeamGeometry(N, a, det_width_factor), dtype, device) for a in per]
