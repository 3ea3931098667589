"""Drop-in for /root/reference/block_6_admm_loop.py (the module block_7_main.py:11 imports).

Accepts that file's keyword surface (:72-84) and runs the full consensus ADMM of
block_6_admm_loop_ver2.py (the skeleton's empty neighbour lists and missing z/y
updates, :119-154, are a reference defect not reproduced).  The returned history has
the ``_ver2`` keys plus this file's ``primal_res`` / ``dual_res`` / ``obj`` (:101-105).

SCS controls map onto the split-Bregman inner solve (CG steps play SCS's iterations,
as block_5_node_problem's ``max_iters`` does):

* ``scs_total_iters`` -> ceil(scs_total_iters / cg_iters) rounds per x-update (unless
  ``tv_iters`` is given explicitly).  The exchange rate is one CG step (one A^T A p) per
  SCS iteration (one KKT matvec in SCS's indirect mode): a modelling choice, not an
  equivalence.  At this file's default (100) that is 20 rounds x 5 CG steps, twice the
  inner work of the ``_ver2`` drop-in's fixed 10 x 5;
* ``scs_chunk_iters`` -> the x-update runs as warm-started chunks of
  ceil(scs_chunk_iters / cg_iters) rounds (:127-146, _scs_solve_in_chunks :14-69);
* ``scs_snapshot_dir`` / ``scs_save_every_chunks`` -> after chunk c (c % every == 0)
  ``{dir}/node_{i}/node_{i}_outer_{k}_chunk_{c}.npy`` with the Fortran-order reshape of
  :58 (+ .png), only for chunked solves, as in the reference (:137-146);
* ``scs_eps`` / ``scs_use_indirect`` / ``scs_alpha`` / ``scs_acceleration`` /
  ``scs_lookback`` / ``scs_scale``: SCS-only, accepted and ignored.
"""
from __future__ import annotations

import math

from admm_hip.admm import run_admm


def _rounds(iters, cg):
    return max(1, math.ceil(int(iters) / cg))


def decentralized_admm(A_dense_list, sinograms, G, Wi_list, Qij_diag_fn,
                       N, lam_tv=0.01, rho=1.0,
                       max_iters=200,
                       eps_pri=1e-3, eps_dual=1e-3,
                       verbose=True,
                       scs_total_iters=100,
                       scs_chunk_iters=None,
                       scs_snapshot_dir=None,
                       scs_use_indirect=True,
                       scs_eps=3e-3, scs_alpha=1.5,
                       scs_acceleration=1, scs_lookback=10, scs_scale=1e-1,
                       scs_save_every_chunks=1,
                       mu=None, tv_iters=None, cg_iters=5, tv_kind="iso", group=None,
                       phantom_true=None, write_params=True):
    del scs_use_indirect, scs_eps, scs_alpha, scs_acceleration, scs_lookback, scs_scale
    cg = int(cg_iters)
    total = int(tv_iters) if tv_iters is not None else _rounds(scs_total_iters, cg)
    chunks = None
    if scs_chunk_iters is not None:
        per = _rounds(scs_chunk_iters, cg)
        chunks = [per] * (total // per) + ([total % per] if total % per else [])
    x, hist = run_admm(A_dense_list, sinograms, G, Wi_list, Qij_diag_fn, N, lam_tv=lam_tv,
                       rho=rho, max_iters=max_iters, eps_pri=eps_pri, eps_dual=eps_dual,
                       verbose=verbose, phantom_true=phantom_true, mu=mu, tv_iters=total,
                       cg_iters=cg, tv_kind=tv_kind, group=group, write_params=write_params,
                       inner_chunks=chunks,
                       chunk_snapshot_dir=scs_snapshot_dir if chunks is not None else None,
                       chunk_save_every=scs_save_every_chunks)
    hist["primal_res"] = hist["primal"]
    hist["dual_res"] = hist["dual"]
    hist["obj"] = hist["obj_total"]
    return x, hist
