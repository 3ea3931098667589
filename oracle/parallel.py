"""Oracle: node x-updates of an ADMM trajectory in parallel processes.  TEST
INFRASTRUCTURE ONLY (see oracle/__init__.py).

The x-updates of one outer iteration are independent (Jacobi: each uses only the
previous z, y -- block_6_admm_loop_ver2.py:81-97), so running them in separate
processes gives exactly the sequential loop's results.

Layout (cheap enough that whole C2/C3 trajectories fit the GPU suite's budget):

* the Joseph CSR matrix and its transpose are built ONCE, in this process, and written as
  ``.npy`` arrays to a scratch directory; every worker reads them into its own memory (no
  per-worker rebuild; private pages keep the SpMVs on the worker's NUMA node);
* node i lives in worker ``i % procs`` for the whole trajectory: its b_i, A^T b_i and
  split-Bregman ``NodeState`` never cross a pipe after ``bind``;
* per iteration a worker receives only its nodes' (q_ij, v_ij) lists and returns only x_i
  and the node's diagnostics.

    with NodePool(N, a, procs=8) as pool:
        oracle.admm.decentralized_admm([pool.A] * V, ..., pool=pool)
"""
from __future__ import annotations

import multiprocessing as mp
import os
import shutil
import tempfile
import time

import numpy as np

_PARTS = ("data", "indices", "indptr")


def _save_csr(M, d, name):
    for p in _PARTS:
        np.save(os.path.join(d, f"{name}_{p}.npy"), getattr(M, p))


def _load_csr(d, name, shape, private=False):
    """The saved CSR matrix, memory-mapped -- or (``private``) read into this process's own
    memory: first-touched by the worker, so on a multi-socket host its pages sit on the worker's
    NUMA node instead of wherever the shared page cache put them (the C3 pool's x-updates ran at
    5.7-7.8 s per node from the shared mapping on the GPU box, against 2.6 s in bench.py's
    private-matrix workers)."""
    import scipy.sparse as sp
    arr = [np.load(os.path.join(d, f"{name}_{p}.npy"), mmap_mode=None if private else "r") for p in _PARTS]
    return sp.csr_matrix(tuple(arr), shape=shape)


def _worker(conn, d, shape):
    from . import node_solver as ns
    A = _load_csr(d, "A", shape, private=True)
    AT = _load_csr(d, "AT", shape[::-1], private=True)
    nodes = {}  # i -> (b_i, A^T b_i, NodeState)
    prm = N = dtype = None
    conn.send("ready")
    while True:
        msg = conn.recv()
        if msg[0] == "stop":
            break
        if msg[0] == "bind":
            _, bs, prm, N, dtype = msg
            nodes = {i: (b, AT @ b, ns.NodeState.zeros(N * N, dtype)) for i, b in bs.items()}
            conn.send("bound")
            continue
        out = []
        t0 = time.perf_counter()
        for i, qv in msg[1]:
            b, Atb, st = nodes[i]
            D, c = ns.assemble(qv, N * N)
            diag = ns.node_update(A, Atb, b, D, c, qv, st, N, prm, dtype=dtype, AT=AT)
            out.append((i, st.x, diag))
        conn.send((out, time.perf_counter() - t0))


class NodePool:
    """``procs`` worker processes sharing one memory-mapped Joseph CSR matrix of
    ``Geometry(N, a)``; nodes are pinned to workers (see the module docstring)."""

    def __init__(self, N, a, procs=None, verbose=False):
        from .geometry import Geometry, joseph_matrix
        self.procs = procs or min(8, os.cpu_count() or 1)
        self.verbose = verbose
        self.A = joseph_matrix(Geometry(N, a))
        self._dir = tempfile.mkdtemp(prefix="oracle_csr_")
        _save_csr(self.A, self._dir, "A")
        _save_csr(self.A.T.tocsr(), self._dir, "AT")
        ctx = mp.get_context("spawn")
        saved = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")}
        for k in saved:
            os.environ[k] = "1"
        try:
            self._conns, self._procs = [], []
            for _ in range(self.procs):
                here, there = ctx.Pipe()
                p = ctx.Process(target=_worker, args=(there, self._dir, self.A.shape), daemon=True)
                p.start()
                self._conns.append(here)
                self._procs.append(p)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        for c in self._conns:
            assert c.recv() == "ready"
        self._t0 = time.perf_counter()
        self._iters = 0

    def bind(self, b_list, prm, N, dtype):
        """Hand every node its sinogram; (re)starts every node from the zero state."""
        for w, c in enumerate(self._conns):
            c.send(("bind", {i: b for i, b in enumerate(b_list) if i % self.procs == w}, prm, N, dtype))
        for c in self._conns:
            assert c.recv() == "bound"
        self._t0 = time.perf_counter()
        self._iters = 0

    def update(self, tasks):
        """tasks = [(i, [(q_ij, v_ij), ...])] -> [(x_i, NodeDiag)] in the order of ``tasks``."""
        per = [[] for _ in self._conns]
        for i, qv in tasks:
            per[i % self.procs].append((i, qv))
        busy = [w for w, t in enumerate(per) if t]
        for w in busy:
            self._conns[w].send(("update", per[w]))
        got, busy_s = {}, []
        t0 = time.perf_counter()
        for w in busy:
            out, dt = self._conns[w].recv()
            busy_s.append(dt)
            for i, x, d in out:
                got[i] = (x, d)
        self._iters += 1
        if self.verbose:
            print(f"oracle iteration {self._iters}: {len(tasks)} node updates, "
                  f"{time.perf_counter() - self._t0:.1f} s since bind (this one {time.perf_counter() - t0:.1f} s; "
                  f"worker compute {min(busy_s):.1f}-{max(busy_s):.1f} s)", flush=True)
        return [got[i] for i, _ in tasks]

    def close(self):
        for c in self._conns:
            try:
                c.send(("stop",))
            except (BrokenPipeError, OSError):
                pass
        for p in self._procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
        shutil.rmtree(self._dir, ignore_errors=True)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
