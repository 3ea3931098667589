"""Drop-in for /root/reference/block_6_admm_loop_ver2.py (the canonical ADMM loop).

Same signature (:15-20) and history keys (:310-326); the node solves and edge
updates run on MI355X (admm_hip.admm.run_admm).  Extra keyword arguments:

* ``mu``        split-Bregman penalty (default 10 * lam_tv)
* ``tv_iters``  split-Bregman rounds per x-update (default 10)
* ``cg_iters``  CG steps per round (default 5)
* ``tv_kind``   "iso" (default) or "aniso"
* ``group``     torch.distributed process group (default: WORLD if initialised)
* ``fusion``    "midpoint" (default; z = (a_i + a_j)/2 as the reference runs, :220-223)
                or "weighted" (z = (W_i a_i + W_j a_j)/(W_i + W_j) with W = Wi_list, the
                form commented out at :221-222 and ADMM_Algo.pdf eq.(2))

* ``inner_tol``  None (default: fixed tv_iters x cg_iters per x-update, deterministic) or
                "reference" (the accept / tighten loop of :100-176: solve to
                eps_try = min(1e-2, eps_target), accept if ||g|| <= eps_target, else
                eps_try /= 5, at most twice; see admm_hip/admm.py)
* ``max_inner_updates``  x-updates per tolerance solve in "reference" mode (default 10)

``max_inner_iters`` is accepted and, as in the reference, unused.
"""
from __future__ import annotations

from admm_hip.admm import run_admm


def decentralized_admm(A_dense_list, sinograms, G, Wi_list, Qij_diag_fn,
                       N, lam_tv=0.01, rho=1.0,
                       max_iters=10, max_inner_iters=100,
                       eps_pri=1e-1, eps_dual=1e-1,
                       verbose=True, snapshot_dir=None,
                       snapshot_every=None, snapshot_div=10, phantom_true=None,
                       mu=None, tv_iters=10, cg_iters=5, tv_kind="iso", group=None,
                       write_params=True, fusion="midpoint", inner_tol=None,
                       max_inner_updates=10):
    """Returns (x_list, history) like block_6_admm_loop_ver2.py:310-326."""
    del max_inner_iters  # accepted but unused, as in the reference (_ver2:17)
    return run_admm(A_dense_list, sinograms, G, Wi_list, Qij_diag_fn, N, lam_tv=lam_tv, rho=rho,
                    max_iters=max_iters, eps_pri=eps_pri, eps_dual=eps_dual, verbose=verbose,
                    snapshot_dir=snapshot_dir, snapshot_every=snapshot_every,
                    snapshot_div=snapshot_div, phantom_true=phantom_true, mu=mu,
                    tv_iters=tv_iters, cg_iters=cg_iters, tv_kind=tv_kind, group=group,
                    write_params=write_params, fusion=fusion, inner_tol=inner_tol,
                    max_inner_updates=max_inner_updates)
