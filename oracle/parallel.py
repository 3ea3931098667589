"""Oracle: node x-updates of one ADMM iteration in parallel processes.  TEST
INFRASTRUCTURE ONLY (see oracle/__init__.py).

The x-updates of one outer iteration are independent (Jacobi: each uses only the
previous z, y -- block_6_admm_loop_ver2.py:81-97), so running them in separate
processes gives exactly the sequential loop's results.  Every worker builds the same
Joseph CSR matrix once (oracle/geometry.py) and serves ``node_update`` tasks; this makes
whole-trajectory oracle runs at 256^2-512^2 (BASELINE C2/C3) take seconds.

    with NodePool(N, a, procs=8) as pool:
        oracle.admm.decentralized_admm([A] * V, ..., node_map=pool.map)
"""
from __future__ import annotations

import multiprocessing as mp
import os

_A = None
_AT = None


def _init(N, a):
    global _A, _AT
    os.environ["OMP_NUM_THREADS"] = "1"
    from .geometry import Geometry, joseph_matrix
    _A = joseph_matrix(Geometry(N, a))
    _AT = _A.T.tocsr()


def _run(task):
    from . import node_solver as ns
    i, b, D, c, qv, st, N, prm, dtype = task
    d = ns.node_update(_A, _AT @ b, b, D, c, qv, st, N, prm, dtype=dtype, AT=_AT)
    return st, d


class NodePool:
    def __init__(self, N, a, procs=None):
        procs = procs or min(8, os.cpu_count() or 1)
        self.pool = mp.get_context("spawn").Pool(procs, initializer=_init, initargs=(N, a))

    def map(self, tasks):
        return self.pool.map(_run, tasks, chunksize=1)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.pool.close()
        self.pool.join()
