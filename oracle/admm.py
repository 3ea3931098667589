"""Oracle: decentralized edge-split ADMM loop.  TEST INFRASTRUCTURE ONLY.

Restates /root/reference/block_6_admm_loop_ver2.py:15-326 with the node solve
of ``node_solver`` (fixed-count split-Bregman + CG instead of CVXPY+SCS):

  * state init x=0, z=0, y=0 (:35-43); b_i = sinograms[i].reshape(-1) (:46)
  * neighbour gather v_ij = z_ij - y_ij,i, q_ij = Qij_diag_fn(i,j) (:85-95)
  * eps_target = 2/(k+1)^1.005, first SCS eps = min(1e-2, eps_target) (:101-108)
  * inner_tol="reference": the accept / tighten loop of :110-176 -- an inner solve to
    eps_try (x-updates until the split-Bregman stationarity residual <= eps_try, at most
    max_inner_updates), accept if ||g|| <= eps_target, else eps_try /= 5, at most two
    tightenings, then force-accept; eps_used = the eps_try of the accepted iterate
  * z_ij = (a_i + a_j)/2 with a = x + y (:210-223); y += x - z (:225-230)
  * fusion="weighted": z_ij = (W_i a_i + W_j a_j)/(W_i + W_j), the form the
    code comments at :216-222 and ADMM_Algo.pdf eq.(2) give
  * r2, s2, per-node attribution, sqrt, stop test (:232-289)
  * history keys (:310-326)

Edge state is kept in the single-y form the device uses: y_e is the dual of
the lower-numbered endpoint a, the other endpoint's dual is -y_e (with y0=0,
y_ij,i + y_ij,j = 0 holds after every update -- SURVEY.md 8a row a7).  Both
ends then evaluate  a_a = x_a + y_e,  a_b = x_b - y_e,  z = (a_a + a_b)/2,
y_e += x_a - z  in that order.  ``edge_update_literal`` restates the
reference's two-dual dict form verbatim for cross-checking.  Weighted fusion
breaks y_ij,i + y_ij,j = 0, so it keeps both duals: y_e (lower endpoint a) and
y2_e (higher endpoint b):  a_a = x_a + y_e,  a_b = x_b + y2_e,
z = (W_a a_a + W_b a_b)/(W_a + W_b),  y_e += x_a - z,  y2_e += x_b - z.
"""
from __future__ import annotations

import math
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import node_solver as ns

HISTORY_KEYS = (
    "primal", "dual", "pri_per_node", "dual_per_node", "obj_per_node", "obj_total",
    "mse_sino_per_node", "mse_sino_total", "img_mse_per_node", "img_mse_total",
    "g_norm_history", "eps_used_history", "eps_target_history",
)
EXTRA_KEYS = ("sb_res_history", "inner_updates_history")
EPS_CAP, CALIB_ALPHA, MAX_TIGHTEN = 1e-2, 1.0, 2  # block_6_admm_loop_ver2.py:106-113


def canonical_edges(G) -> list[tuple[int, int]]:
    """Edges as (min, max) in ``G.edges()`` order (block_6_admm_loop_ver2.py:39-40)."""
    return [(min(i, j), max(i, j)) for i, j in G.edges()]


def eps_target(k: int) -> float:
    return 2.0 / ((k + 1) ** 1.005)  # block_6_admm_loop_ver2.py:101-103


def edge_update_literal(G, x, y, z, Wi_list=None):
    """Verbatim restatement of block_6_admm_loop_ver2.py:210-230 (two duals per edge).

    With ``Wi_list`` the numerator/denominator are the weighted ones the
    reference leaves commented out at :221-222.
    """
    new_z = {}
    for i, j in G.edges():
        key = (min(i, j), max(i, j))
        a_i = x[i] + y[(key[0], key[1], i)]
        a_j = x[j] + y[(key[0], key[1], j)]
        if Wi_list is None:
            new_z[key] = (a_i + a_j) / 2.0
        else:
            Wi, Wj = Wi_list[i], Wi_list[j]
            new_z[key] = (Wi * a_i + Wj * a_j) / (Wi + Wj)
    new_y = {}
    for i, j in G.edges():
        key = (min(i, j), max(i, j))
        new_y[(key[0], key[1], i)] = y[(key[0], key[1], i)] + x[i] - new_z[key]
        new_y[(key[0], key[1], j)] = y[(key[0], key[1], j)] + x[j] - new_z[key]
    return new_z, new_y


class _Serialized:
    """An operator whose products run one at a time (a lock shared by every node's operator
    and adjoint): the GPU RayTransform of the operator-level oracle shares one context --
    and its scratch buffers -- per geometry, so concurrent node threads must not interleave
    its launches.  Only the products serialize; the float64 vector algebra runs in parallel."""

    def __init__(self, op, lock, T=None):
        self.op, self.lock, self._T = op, lock, T
        self.shape = op.shape

    @property
    def T(self):
        if self._T is None:
            self._T = _Serialized(self.op.T, self.lock, self)
        return self._T

    def __matmul__(self, x):
        with self.lock:
            return self.op @ x


def decentralized_admm(ops, sinograms, G, Qij_diag_fn, N, lam_tv=0.01, rho=1.0,
                       max_iters=10, eps_pri=1e-1, eps_dual=1e-1, phantom_true=None,
                       mu=None, tv_iters=10, cg_iters=5, tv_kind="iso",
                       dtype=np.float64, node_subset=None, fusion="midpoint", Wi_list=None,
                       inner_tol=None, max_inner_updates=10, pool=None, threads=None):
    """Oracle ADMM.  ``ops`` = list of scipy sparse matrices (one per node).

    Returns (x_list, history) with the reference's history keys.  With
    ``node_subset`` only those nodes' x-updates run (the others keep x=0); used
    only to time a bounded CPU sample.  ``fusion="weighted"`` needs ``Wi_list``.
    ``pool`` (fixed-count mode only; oracle/parallel.NodePool) runs the iteration's
    independent node updates in worker processes that hold each node's state for the whole
    trajectory: ``pool.bind(b, params, N, dtype)`` once, then ``pool.update([(i, qv)])`` ->
    [(x_i, diag)] per iteration (Jacobi order, so results equal the sequential loop).
    ``threads`` (fixed-count mode only; the operator-level oracle over GPU RayTransforms) runs
    an iteration's node updates in that many threads, the operator products serialized
    (``_Serialized``): the same per-node arithmetic, so the same results.
    """
    if threads is not None and (inner_tol is not None or pool is not None):
        raise ValueError("threads runs fixed-count updates without a pool only")
    if threads is not None and threads > 1:
        lock = threading.Lock()
        ops = [_Serialized(A, lock) for A in ops]
    if pool is not None and inner_tol is not None:
        raise ValueError("pool runs fixed-count updates only")
    if fusion not in ("midpoint", "weighted"):
        raise ValueError("fusion must be 'midpoint' or 'weighted'")
    weighted = fusion == "weighted"
    if weighted:
        if Wi_list is None:
            raise ValueError("weighted fusion needs Wi_list")
        W = [np.asarray(w, dtype=np.float64).reshape(-1) for w in Wi_list]
    V = len(ops)
    n = N * N
    mu = (10.0 * lam_tv if mu is None else mu)
    prm = ns.NodeParams(rho=rho, lam=lam_tv, mu=mu, tv_iters=tv_iters, cg_iters=cg_iters,
                        tv_kind=tv_kind)
    edges = canonical_edges(G)
    b = [np.asarray(s, dtype=np.float64).reshape(-1) for s in sinograms]
    # scipy matrices; any object with @ and .T (e.g. the GPU RayTransform, used by the
    # full-size tests as an operator-level oracle: this loop's float64 vector algebra
    # around a projector that is itself checked against joseph_matrix)
    if pool is None:
        ATs = [A.T.tocsr() if hasattr(A.T, "tocsr") else A.T for A in ops]
        Atb = [ATs[i] @ b[i] for i in range(V)]
    else:
        pool.bind(b, prm, N, dtype)
    states = [ns.NodeState.zeros(n, dtype) for _ in range(V)]
    y = {e: np.zeros(n) for e in edges}
    z = {e: np.zeros(n) for e in edges}
    y2 = {e: np.zeros(n) for e in edges} if weighted else None
    nbrs = {i: list(G.neighbors(i)) for i in range(V)}
    if inner_tol not in (None, "reference"):
        raise ValueError("inner_tol must be None or 'reference'")
    hist = {k: [] for k in HISTORY_KEYS + EXTRA_KEYS}
    ph = None
    if phantom_true is not None:
        ph = np.asarray(phantom_true, dtype=np.float64).reshape(-1)
    x = [np.zeros(n) for _ in range(V)]
    for k in range(max_iters):
        obj_i = np.zeros(V)
        g_i = np.zeros(V)
        mse_i = np.zeros(V)
        sb_i = np.zeros(V)
        # eps_used: the tolerance the accepted iterate was solved to (NaN for fixed counts)
        eu_i = np.full(V, min(EPS_CAP, CALIB_ALPHA * eps_target(k)) if inner_tol else np.nan)
        nu_i = np.zeros(V, dtype=np.int64)
        et = eps_target(k)
        todo = range(V) if node_subset is None else node_subset
        tasks = []
        for i in todo:
            qv = []
            for j in nbrs[i]:
                e = (min(i, j), max(i, j))
                yi = y[e] if i == e[0] else (y2[e] if weighted else -y[e])
                qv.append((np.asarray(Qij_diag_fn(i, j), dtype=np.float64), z[e] - yi))
            if pool is not None or (threads is not None and threads > 1):
                tasks.append((i, qv))
                continue
            D, c = ns.assemble(qv, n)
            d = ns.node_update(ops[i], Atb[i], b[i], D, c, qv, states[i], N, prm, dtype=dtype,
                               AT=ATs[i])
            nu_i[i] = 1
            if inner_tol == "reference":
                eps_try, tries = eu_i[i], 0
                while True:
                    while d.sb_res > eps_try and nu_i[i] < (tries + 1) * max_inner_updates:
                        d = ns.node_update(ops[i], Atb[i], b[i], D, c, qv, states[i], N, prm,
                                           dtype=dtype, AT=ATs[i])
                        nu_i[i] += 1
                    if d.g_norm <= et or tries >= MAX_TIGHTEN:
                        break
                    tries += 1
                    eps_try /= 5.0
                eu_i[i] = eps_try
            obj_i[i] = d.obj
            sb_i[i] = d.sb_res
            g_i[i] = d.g_norm
            mse_i[i] = d.mse_sino
        if threads is not None and threads > 1 and tasks:
            def update(task):  # one node's x-update (its own state; products serialized)
                i, qv = task
                D, c = ns.assemble(qv, n)
                return ns.node_update(ops[i], Atb[i], b[i], D, c, qv, states[i], N, prm, dtype=dtype, AT=ATs[i])

            with ThreadPoolExecutor(threads) as ex:
                done = list(ex.map(update, tasks))
            for (i, _), d in zip(tasks, done):
                nu_i[i] = 1
                obj_i[i], sb_i[i], g_i[i], mse_i[i] = d.obj, d.sb_res, d.g_norm, d.mse_sino
        if pool is not None:
            for (i, _), (xi, d) in zip(tasks, pool.update(tasks)):
                states[i].x = xi
                nu_i[i] = 1
                obj_i[i], sb_i[i], g_i[i], mse_i[i] = d.obj, d.sb_res, d.g_norm, d.mse_sino
        x = [st.x.astype(np.float64) for st in states]
        hist["g_norm_history"].append(g_i)
        hist["eps_used_history"].append(eu_i)
        hist["sb_res_history"].append(sb_i)
        hist["inner_updates_history"].append(nu_i)
        hist["eps_target_history"].append(np.full(V, et))
        hist["mse_sino_per_node"].append(mse_i)
        hist["mse_sino_total"].append(float(np.sum(mse_i)))
        if ph is not None:
            img = np.array([float((xi - ph) @ (xi - ph)) for xi in x])
        else:
            img = np.full(V, np.nan)
        hist["img_mse_per_node"].append(img)
        hist["img_mse_total"].append(float(np.sum(img)))
        r2 = 0.0
        s2 = 0.0
        pri = np.zeros(V)
        dua = np.zeros(V)
        for (a_, b_) in edges:
            e = (a_, b_)
            aa = x[a_] + y[e]
            if weighted:
                ab = x[b_] + y2[e]
                zn = (W[a_] * aa + W[b_] * ab) / (W[a_] + W[b_])
                y2[e] = y2[e] + x[b_] - zn
            else:
                ab = x[b_] - y[e]
                zn = (aa + ab) * 0.5
            y[e] = y[e] + x[a_] - zn
            ra = x[a_] - zn
            rb = x[b_] - zn
            dz = zn - z[e]
            z[e] = zn
            ra2 = float(ra @ ra)
            rb2 = float(rb @ rb)
            dz2 = float(dz @ dz)
            r2 += ra2 + rb2
            pri[a_] += ra2
            pri[b_] += rb2
            s2 += rho * rho * dz2
            dua[a_] += rho * rho * dz2
            dua[b_] += rho * rho * dz2
        pn, dn = math.sqrt(r2), math.sqrt(s2)
        hist["primal"].append(pn)
        hist["dual"].append(dn)
        hist["obj_per_node"].append(obj_i)
        hist["obj_total"].append(float(np.sum(obj_i)))
        hist["pri_per_node"].append(np.sqrt(pri))
        hist["dual_per_node"].append(np.sqrt(dua))
        if pn < eps_pri and dn < eps_dual:
            break
    return x, hist
