"""GPU parity of the hot forward kernel (k_fwdg + k_fwd_combine) at the BASELINE sizes.

``RayTransform @ X`` with 1-8 images runs the hot path's own grouped forward
projector (admm_project_fwd packs the images into the node-interleaved sample
layout, VB = 1/2/4/8 by image count).  The oracle is the float64 Joseph CSR
matrix of oracle/geometry.py restricted to a handful of angles per case (the
full matrix is ~2.4 GB at 1024^2 and ~10 GB at 2048^2): both sides of the
45-degree case switch, the first/last angles and the quarter points.  All
angle-group plans (64-ray chunks / aligned per segment and angle / aligned per segment and
chunk, each with and without rays clipped to the segment; ADMM_FWD_PLAN 0-5) are checked.

Tolerance (relative Frobenius over the checked rows): float32 samples 4e-6
(sums of up to 2N float32 products per ray in 8 segment partials),
float64 samples 1e-12.
"""
import os

import numpy as np
import pytest
import torch

from admm_hip.geometry import ParallelBeamGeometry, RayTransform
from oracle.geometry import Geometry, joseph_matrix, shepp_logan

pytestmark = pytest.mark.gpu

TOL = {"float32": 4e-6, "float64": 1e-12}


def _angle_subset(a):
    """First / last, quarter points, and the two angles around 45 and 135 degrees."""
    th = (np.arange(a) + 0.5) * np.pi / a
    caseA = np.abs(np.cos(th)) >= np.abs(np.sin(th))
    sw = [t for t in range(1, a) if caseA[t] != caseA[t - 1]]
    sel = {0, a - 1, a // 4, a // 2, (3 * a) // 4}
    for t in sw:
        sel.update((t - 1, t))
    return sorted(sel)


def _images(N, k, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((k, N * N))
    X[0] = shepp_logan(N, 2).ravel()
    return X


def _check(N, a, dtype, k, plan, seed):
    os.environ["ADMM_FWD_PLAN"] = str(plan)
    try:
        op = RayTransform(ParallelBeamGeometry(N, a), dtype)
        tdt = torch.float64 if dtype == "float64" else torch.float32
        X = _images(N, k, seed)
        Xt = torch.as_tensor(X, dtype=tdt)
        Y = (op @ Xt.cuda()).double().cpu().numpy().reshape(k, a, N)
        torch.cuda.synchronize()
    finally:
        os.environ.pop("ADMM_FWD_PLAN", None)
    sel = _angle_subset(a)
    A = joseph_matrix(Geometry(N, a), angles=sel)
    Xs = Xt.double().numpy()
    worst = 0.0
    for v in range(k):
        ref = (A @ Xs[v]).reshape(len(sel), N)
        got = Y[v][sel]
        e = float(np.linalg.norm(got - ref) / np.linalg.norm(ref))
        worst = max(worst, e)
    assert worst < TOL[dtype], (N, a, dtype, k, plan, worst)
    return worst


@pytest.mark.parametrize("N", [256, 512, 1024])
@pytest.mark.parametrize("plan", [0, 1, 2, 3, 4, 5])
def test_grouped_forward_vb8_float32(cuda, N, plan):
    """8 images = the benchmark's k_fwdg<float, 8> instance (C2, C3/bench, C4 sizes)."""
    _check(N, 96, "float32", 8, plan, seed=N + plan)


@pytest.mark.parametrize("k", [1, 2, 3])
def test_grouped_forward_narrow_batches(cuda, k):
    """VB = 1, 2, 4 instances (single-node drop-in, 2-node and 3-4-node shards)."""
    _check(512, 96, "float32", k, 1, seed=7 * k)


@pytest.mark.parametrize("plan", [0, 1, 2, 3, 4, 5])
def test_grouped_forward_2048_float64(cuda, plan):
    """C5 size and precision: 2048^2, 96 angles per node, float64 samples, 8 images."""
    _check(2048, 96, "float64", 8, plan, seed=2048 + plan)


def test_grouped_forward_default_angles(cuda):
    """C1-style per-node angle counts (180 total over 4 nodes = 45: one angle at pi/2)."""
    _check(64, 45, "float32", 4, 1, seed=45)
    _check(64, 45, "float64", 4, 0, seed=46)
    _check(64, 45, "float32", 4, 2, seed=47)
    _check(64, 45, "float64", 4, 5, seed=48)


def _check_adjoint(N, a, dtype, k, seed, tol):
    """A^T y with y nonzero only on the sampled angles, against the Joseph CSR matrix of those
    angles transposed (k_back's tap loop -- every mode shares it -- at full size)."""
    op = RayTransform(ParallelBeamGeometry(N, a), dtype)
    tdt = torch.float64 if dtype == "float64" else torch.float32
    sel = _angle_subset(a)
    rng = np.random.default_rng(seed)
    Y = np.zeros((k, a, N))
    Y[:, sel, :] = rng.standard_normal((k, len(sel), N))
    Yt = torch.as_tensor(Y.reshape(k, a * N), dtype=tdt)
    X = (op.T @ Yt.cuda()).double().cpu().numpy()
    torch.cuda.synchronize()
    A = joseph_matrix(Geometry(N, a), angles=sel)
    Ys = Yt.double().numpy().reshape(k, a, N)[:, sel, :].reshape(k, -1)
    worst = max(float(np.linalg.norm(X[v] - A.T @ Ys[v]) / np.linalg.norm(A.T @ Ys[v])) for v in range(k))
    assert worst < tol, (N, a, dtype, worst)
    return worst


def test_adjoint_1024_float32(cuda):
    """C4 size: A^T at 1024^2, 96 angles, float32 samples (k_back was pinned at
    <= 128^2 only; the C4 operator-level oracle uses this A^T)."""
    _check_adjoint(1024, 96, "float32", 2, 11, 4e-6)


def test_adjoint_2048_float64(cuda):
    """C5 size and precision: A^T at 2048^2, 96 angles, float64 samples."""
    _check_adjoint(2048, 96, "float64", 1, 12, 1e-12)


def _bound_plans(N, dtype):
    """The forward plans of an 8-node batch bound at N^2 (admm_fwd_plan_info)."""
    import networkx as nx
    from admm_hip.data import make_precisions, make_sinograms
    from admm_hip.plan import make_plan
    from admm_hip.solver import NodeBatch, make_operators
    ops = make_operators(N, 8, angles_total=96 * 8, dtype=dtype, device=0)
    plan = make_plan(nx.cycle_graph(8), 8, 1, 0)
    ph = shepp_logan(N)
    sinos = dict(zip(plan.local_nodes, make_sinograms(ops, ph, 0.005, seed=1)))
    _, Q = make_precisions(ops)
    nb = NodeBatch(ops[0].geom, dtype, plan, sinos, Q, 2.0, 0.02, 0.2, 10, 5, "iso", ph, 0)
    return {p["plan"]: p for p in nb.fwd_plans()}


def test_planner_picks_chunk_aligned_plan_for_large_images(cuda):
    """At 2048^2 the per-(segment, angle) alignment lets 64-ray chunks far from the detector
    centre drift apart (the rays' spacing differs between a group's angles), so its groups
    shrink; the chunk-aligned plan stages half the row pixels in fewer blocks and is bound
    (1141 vs 1439 us per float64 launch, profiles/r3_forward_plans.jsonl).  At 512^2 the
    64-ray plan keeps two blocks per CU and stays bound."""
    p = _bound_plans(2048, "float64")
    assert p[5]["active"], p  # chunk-aligned, rays clipped to each segment
    assert p[2]["staged_px"] < 0.6 * p[1]["staged_px"] and p[2]["blocks"] < p[1]["blocks"], p
    assert p[5]["staged_px"] < p[2]["staged_px"] and p[5]["blocks"] < p[2]["blocks"], p
    p = _bound_plans(512, "float32")
    act = [q for q in p.values() if q["active"]]
    assert len(act) == 1 and act[0]["blocks"] <= 512, p  # one round: <= 2 blocks per CU
