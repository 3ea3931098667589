"""GPU: mirror mode of the forward projector (kernels.hpp k_fwdg MIRROR; the float32 default,
ADMM_FWD_MIRROR=0 / 1 forces it off / on).

Angle a-1-t projects I as angle t projects flipud(I) (tests/test_oracle.py::
test_mirror_symmetry_of_the_joseph_operator), so a batch projects virtual images -- its real
nodes at (i, j) and at (N-1-i, j) -- over half the angles, 8 float32 lanes per tap even for a
4-node batch.  Checked: whole ADMM trajectories against the float64 oracle at every node-
interleave width (1e-5 float32 / 1e-9 float64 samples); a node's result bitwise independent
of its batch's size (the mode depends on the geometry only); odd angle counts keep the
direct projection.
"""
import networkx as nx
import numpy as np
import pytest
import torch

from admm_hip.data import make_precisions, make_sinograms, shepp_logan
from admm_hip.solver import make_operators
from block_6_admm_loop_ver2 import decentralized_admm
from oracle import admm as oadmm
from oracle.geometry import Geometry, joseph_matrix

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def _run(N, V, a_per, dtype, iters=3, graph="ring"):
    ops = make_operators(N, V, a_per * V, dtype=dtype, device=0)
    ph = shepp_logan(N)
    sinos = make_sinograms(ops, ph, 0.005, seed=1000)
    Wi, Q = make_precisions(ops)
    G = nx.cycle_graph(V) if graph == "ring" and V > 2 else nx.path_graph(V) if graph == "ring" else nx.empty_graph(V)
    x, h = decentralized_admm(ops, sinos, G, Wi, Q, N, lam_tv=0.02, rho=2.0, max_iters=iters, eps_pri=0.0,
                              eps_dual=0.0, verbose=False, phantom_true=ph.numpy(), write_params=False,
                              tv_iters=4, cg_iters=3)
    torch.cuda.synchronize()
    return ops, ph, sinos, Q, G, np.stack(x), h


@pytest.mark.parametrize("dtype,V,mode,N", [("float32", 1, "1", 48), ("float32", 2, "1", 48), ("float32", 4, "1", 48),
                                            ("float32", 8, "1", 48), ("float32", 12, "1", 48), ("float64", 1, "1", 48),
                                            ("float64", 2, "1", 48), ("float64", 4, "1", 48),
                                            ("float32", 4, "0", 48), ("float32", 12, "0", 48),
                                            ("float32", 1, "1", 47), ("float32", 4, "1", 47), ("float32", 8, "1", 47),
                                            ("float64", 2, "1", 47)])
def test_mirror_trajectory_matches_oracle(cuda, monkeypatch, dtype, V, mode, N):
    """mode "1": mirror mode at every node-interleave width; "0": the direct projection.  Odd
    N (47): the middle row pairs with itself in the back projectors' pixel pairs."""
    monkeypatch.setenv("ADMM_FWD_MIRROR", mode)
    a = 24
    ops, ph, sinos, Q, G, x, h = _run(N, V, a, dtype)
    A = joseph_matrix(Geometry(N, a))
    xo, ho = oadmm.decentralized_admm([A] * V, [s.double().cpu().numpy() for s in sinos], G, Q, N, lam_tv=0.02,
                                      rho=2.0, max_iters=3, eps_pri=0.0, eps_dual=0.0, phantom_true=ph.numpy(),
                                      tv_iters=4, cg_iters=3)
    tol = 1e-5 if dtype == "float32" else 1e-9
    errs = {"x": rel(x, np.stack(xo)), "mse_sino": rel(np.stack(h["mse_sino_per_node"]),
                                                       np.stack(ho["mse_sino_per_node"]))}
    if V > 1:
        errs.update(primal=rel(h["primal"], ho["primal"]), dual=rel(h["dual"], ho["dual"]))
    print(dtype, V, {k: f"{v:.2e}" for k, v in errs.items()})
    assert all(v < tol for v in errs.values()), errs


@pytest.mark.parametrize("dtype,mode,N", [("float32", "1", 40), ("float64", "1", 40), ("float32", "0", 40),
                                         ("float32", "1", 47)])
def test_mirror_result_independent_of_batch_size(cuda, monkeypatch, dtype, mode, N):
    """Node 0 of an edgeless graph (its x-update sees only its own data) in batches of 1, 2,
    3, 4, 8 nodes -- every node-interleave width and both staging paths (LDS-DMA and the
    register path of the narrow widths) -- bitwise the same image and statistics (mirror
    mode, and the direct projection; odd N: the self-paired middle row)."""
    monkeypatch.setenv("ADMM_FWD_MIRROR", mode)
    res = {}
    for V in (1, 2, 3, 4, 8):
        _, _, _, _, _, x, h = _run(N, V, 16, dtype, iters=2, graph="empty")
        res[V] = (x[0], np.stack(h["mse_sino_per_node"])[:, 0], np.stack(h["obj_per_node"])[:, 0])
    for V, r in res.items():
        assert np.array_equal(r[0], res[1][0]), V
        assert np.array_equal(r[1], res[1][1]) and np.array_equal(r[2], res[1][2]), V


def test_mirror_is_the_direct_projection_to_rounding(cuda, monkeypatch):
    """Mirror mode against the direct projection of all angles on the same problem: the same
    iteration up to float32 rounding of the geometry (1e-6); odd angle counts (no mirror
    symmetry in the angle set) keep the direct path bit for bit."""
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("ADMM_FWD_MIRROR", mode)
        out[mode] = _run(48, 4, 24, "float32")[5]
    assert rel(out["1"], out["0"]) < 1e-6
    for mode in ("0", "1"):
        monkeypatch.setenv("ADMM_FWD_MIRROR", mode)
        out["odd" + mode] = _run(48, 4, 23, "float32")[5]
    assert np.array_equal(out["odd0"], out["odd1"])


def test_default_mode_by_sample_type(cuda, monkeypatch):
    """Unset ADMM_FWD_MIRROR: mirror mode for float32 samples (every batch width, 16-byte real
    vectors), the direct projection for float64; odd angle counts never mirror."""
    from admm_hip.plan import make_plan
    from admm_hip.solver import NodeBatch
    monkeypatch.delenv("ADMM_FWD_MIRROR", raising=False)
    for dtype, V, a, want, vb in [("float32", 8, 24, True, 4), ("float32", 3, 24, True, 4),
                                  ("float32", 8, 23, False, 8), ("float64", 4, 24, False, 4)]:
        ops = make_operators(40, V, a * V, dtype=dtype, device=0)
        ph = shepp_logan(40)
        plan = make_plan(nx.cycle_graph(V), V)
        sinos = dict(zip(plan.local_nodes, make_sinograms(ops, ph, 0.005, seed=3)))
        _, Q = make_precisions(ops)
        nb = NodeBatch(ops[0].geom, dtype, plan, sinos, Q, 2.0, 0.02, 0.2, 3, 3, "iso", ph, 0)
        assert nb.mirror == want and nb.ctx_vb == vb, (dtype, V, a, nb.mirror, nb.ctx_vb)


@pytest.mark.parametrize("dtype,V,N", [("float32", 5, 64), ("float32", 16, 128), ("float32", 4, 47),
                                       ("float32", 8, 47), ("float64", 2, 48)])
def test_projector_block_shapes_bitwise(cuda, monkeypatch, dtype, V, N):
    """The mirror back projector's H mode stages its sinogram windows by LDS-DMA into two
    chunk buffers (kernels.hpp k_back_mirror, DMA), and where the grid fills the chip runs two
    lane blocks per block (k_back_mirror_2); ADMM_BK_STAGING at context creation selects
    "dma1" (one lane block per block), "reg" (register-staged windows) or "dma2" (two lane
    blocks wherever they pair up).  The same bins land in LDS and every lane block's taps read
    them in the same order: whole trajectories bitwise equal (5 nodes = a full and a one-node
    lane block; 16 nodes = four lane blocks; odd N; float64 keeps one lane block).  The forward
    projector likewise with one or two virtual chunks per block (ADMM_FWD_CPB=1 / 2, k_fwdg CPB)."""
    monkeypatch.setenv("ADMM_FWD_MIRROR", "1")
    runs = []
    for staging, fcpb in (("dma1", "1"), ("reg", "1"), ("dma2", "2")):
        monkeypatch.setenv("ADMM_BK_STAGING", staging)
        monkeypatch.setenv("ADMM_FWD_CPB", fcpb)
        _, _, _, _, _, x, h = _run(N, V, 24, dtype)
        runs.append((x, {k: np.asarray(h[k]) for k in ("primal", "dual", "obj_total", "mse_sino_total",
                                                       "g_norm_history")}))
    (x0, h0) = runs[0]
    for x1, h1 in runs[1:]:
        assert np.array_equal(x0, x1), float(np.max(np.abs(x0 - x1)))
        for k in h0:
            assert np.array_equal(h0[k], h1[k]), k
