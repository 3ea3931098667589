"""GPU: nodes with different operators (admm_hip/groups.py) against the float64 oracle.

The reference's own data setup gives nodes unequal angle counts: ``max(180, 3N)`` angles
split with the remainder on the first nodes (/root/reference/block_2_load_odl_data.py:31-38),
e.g. its driver defaults N=64, 5 nodes (block_7_main_ver3.py:334-335) -> 39/39/38/38/38.
A saved ``A_dense_list`` may hold matrices of different row counts.  Each
distinct operator is one device batch; edges between batches are held by both.

Tolerance (north star): images and primal / dual trajectories <= 1e-5 relative Frobenius
with float32 samples.
"""
import networkx as nx
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from admm_hip.data import make_precisions, make_sinograms, shepp_logan
from admm_hip.geometry import split_angles
from admm_hip.solver import make_operators
from block_6_admm_loop_ver2 import decentralized_admm
from oracle import admm as oadmm
from oracle.geometry import Geometry, joseph_matrix

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def _check(x, h, xo, ho, tol=1e-5):
    errs = {"x": rel(np.stack(x), np.stack(xo)), "primal": rel(h["primal"], ho["primal"]),
            "dual": rel(h["dual"], ho["dual"]), "mse": rel(h["mse_sino_total"], ho["mse_sino_total"]),
            "obj": rel(h["obj_total"], ho["obj_total"])}
    print({k: f"{v:.2e}" for k, v in errs.items()})
    assert max(errs.values()) < tol, errs


@pytest.mark.parametrize("fusion", ["midpoint", "weighted"])
def test_reference_default_angle_split_matches_oracle(cuda, fusion):
    N, V = 64, 5
    per = split_angles(max(180, 3 * N), V)
    assert per == [39, 39, 38, 38, 38]
    ops = make_operators(N, V, device=0)
    assert [A.geom.n_angles for A in ops] == per
    ph = shepp_logan(N)
    sinos = make_sinograms(ops, ph, 0.005, seed=1000)
    Wi, Q = make_precisions(ops)
    G = nx.cycle_graph(V)
    kw = dict(lam_tv=0.02, rho=2.0, max_iters=4, eps_pri=0.0, eps_dual=0.0, phantom_true=ph.numpy(),
              fusion=fusion)
    x, h = decentralized_admm(ops, sinos, G, Wi, Q, N, verbose=False, write_params=False, **kw)
    As = {a: joseph_matrix(Geometry(N, a)) for a in set(per)}
    xo, ho = oadmm.decentralized_admm([As[a] for a in per], [s.double().cpu().numpy() for s in sinos],
                                      G, Q, N, Wi_list=Wi, **kw)
    _check(x, h, xo, ho)


def test_matrices_of_different_row_counts_match_oracle(cuda):
    """A_dense_list of three different matrices (33 / 32 / 31 angles at 32^2, CSR and
    dense mixed): three device batches, complete graph."""
    N = 32
    mats = [joseph_matrix(Geometry(N, a)).tocsr() for a in (33, 32, 31)]
    ph = shepp_logan(N).numpy().ravel()
    rng = np.random.default_rng(5)
    sinos = [(A @ ph + 0.005 * rng.standard_normal(A.shape[0])).astype(np.float32) for A in mats]
    lst = [mats[0], mats[1].toarray(), sp.csc_matrix(mats[2])]
    Wi, Q = make_precisions(lst)
    G = nx.complete_graph(3)
    kw = dict(lam_tv=0.02, rho=2.0, max_iters=4, eps_pri=0.0, eps_dual=0.0, phantom_true=ph)
    x, h = decentralized_admm(lst, sinos, G, Wi, Q, N, verbose=False, write_params=False, **kw)
    xo, ho = oadmm.decentralized_admm(mats, [s.astype(np.float64) for s in sinos], G, Q, N, **kw)
    _check(x, h, xo, ho)
    torch.cuda.synchronize()
