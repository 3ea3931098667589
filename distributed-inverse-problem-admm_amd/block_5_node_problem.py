"""Drop-in for /root/reference/block_5_node_problem.py.

``build_node_problem(Ai, bi, rho, neighbor_terms, N, lam_tv, Qij_terms)``
returns ``(xi, prob)`` duck-typing the CVXPY objects the reference's callers
use (block_6_admm_loop_ver2.py:97-135, test_block5_with_aggregate.py:59-73):

* ``prob.solve(**kw)``  -- runs the x-update of eq.(1) on the GPU (fixed-count
  split-Bregman + CG, warm-started from the previous solve).  CVXPY/SCS keywords
  (solver, eps, warm_start, verbose, acceleration_lookback, use_indirect, ...)
  are accepted and ignored; ``max_iters`` sets the CG budget
  (tv_iters = ceil(max_iters / cg_iters)); ``tv_iters`` / ``cg_iters`` /
  ``mu`` / ``tv_kind`` may be given explicitly.
* ``prob.value``, ``prob.status``, ``prob.solver_stats.num_iters``
* ``xi.value``  -- (n,) float64 numpy array

The objective is 0.5||Ai x - bi||^2 + lam_tv TV(x) + sum_j rho/2 ||x - v_ij||^2_Qij
(:21-29), with textbook isotropic TV (the reference's
CVXPY atom mis-pairs its differences; documented deviation).
"""
from __future__ import annotations

import math
from types import SimpleNamespace

import numpy as np
import torch

from admm_hip import _lib
from admm_hip.admm import DEFAULT_MU_FACTOR
from admm_hip.geometry import RayTransform
from admm_hip.matrix import MatrixOperator, as_operators
from admm_hip.plan import ShardPlan
from admm_hip.solver import NodeBatch


class _Variable:
    def __init__(self, n):
        self.shape = (n,)
        self.value = None


def _star_plan(deg: int) -> ShardPlan:
    """Node 0 (local) with deg virtual neighbours 1..deg (halo rows, never updated)."""
    edges = [(0, j) for j in range(1, deg + 1)]
    P = ShardPlan(V_total=deg + 1, world=1, rank=0, edges=edges, ranges=[(0, 1)])
    P.local_nodes = [0]
    P.halo_nodes = list(range(1, deg + 1))
    P.xrow = {g: g for g in range(deg + 1)}
    P.stored_edges = list(range(deg))
    P.edge_a_row = [0] * deg
    P.edge_b_row = list(range(1, deg + 1))
    P.owned_edge = [True] * deg
    P.inc_off = [0, deg]
    P.inc_edge = list(range(deg))
    P.inc_nbr = list(range(1, deg + 1))
    P.inc_sign = [1] * deg
    return P


class _Problem:
    def __init__(self, Ai, bi, rho, neighbor_terms, N, lam_tv, Qij_terms, xi):
        if not isinstance(Ai, (RayTransform, MatrixOperator)):
            Ai = as_operators([Ai], N=N)[0]  # a matrix (dense / scipy.sparse): explicit-matrix operator
        if Ai._adjoint:
            raise TypeError("Ai is an adjoint view")
        if Ai.geom.N != N:
            raise ValueError(f"N={N} does not match the operator's N={Ai.geom.N}")
        if len(neighbor_terms) != len(Qij_terms):
            raise ValueError("neighbor_terms and Qij_terms differ in length")
        self.A, self.b, self.rho, self.N, self.lam = Ai, bi, float(rho), N, float(lam_tv)
        self.v = list(neighbor_terms)
        self.q = list(Qij_terms)
        self.xi = xi
        self.nb = None
        self.cfg = None
        self.value = None
        self.status = None
        self.solver_stats = SimpleNamespace(num_iters=None, solver_name="admm_hip")

    def _build(self, tv_iters, cg_iters, mu, tv_kind):
        deg = len(self.v)
        qs = self.q
        qfn = lambda i, j: qs[j - 1]  # noqa: E731
        nb = NodeBatch(self.A.geom, self.A.dtype, _star_plan(deg), [self.b], qfn, self.rho,
                       self.lam, mu, tv_iters, cg_iters, tv_kind, None, self.A.device,
                       derive_z=False)  # the targets v_ij are the caller's: stored as z, y = 0
        for e, v in enumerate(self.v):
            nb.z[e].copy_(torch.as_tensor(np.asarray(v) if not isinstance(v, torch.Tensor) else v)
                          .reshape(-1).to(device=nb.dev, dtype=torch.float64))
        if self.xi.value is not None:
            nb.x_ext[0].copy_(torch.as_tensor(np.asarray(self.xi.value, dtype=np.float64)))
        self.nb = nb
        self.cfg = (tv_iters, cg_iters, mu, tv_kind)

    def solve(self, *args, max_iters=None, tv_iters=None, cg_iters=None, mu=None,
              tv_kind="iso", **ignored):
        cg = int(cg_iters) if cg_iters is not None else 5
        if tv_iters is None:
            tv_iters = 10 if max_iters is None else max(1, math.ceil(int(max_iters) / cg))
        if mu is None:
            mu = DEFAULT_MU_FACTOR * self.lam if self.lam > 0 else 1e-12
        cfg = (int(tv_iters), cg, float(mu), tv_kind)
        if self.nb is None or self.cfg != cfg:
            self._build(*cfg)
        self.nb.node_update()
        st = self.nb.node_stats[0].to("cpu").numpy()
        self.value = 0.5 * st[0] + self.lam * st[2] + st[3]
        self.status = "optimal_inaccurate"  # fixed iteration budget, no tolerance test
        self.solver_stats.num_iters = cfg[0] * cfg[1]
        self.xi.value = self.nb.x_ext[0].to("cpu").numpy().copy()
        self.g_norm = float(math.sqrt(st[1]))
        return self.value


def build_node_problem(Ai, bi, rho, neighbor_terms, N, lam_tv, Qij_terms):
    """(xi, prob) for node objective eq.(1) -- block_5_node_problem.py:6-32."""
    xi = _Variable(Ai.shape[1])
    prob = _Problem(Ai, bi, rho, neighbor_terms, N, lam_tv, Qij_terms, xi)
    return xi, prob
