"""CPU: bench.py's launch decision (driver contract), its CPU leg and the C4 graph fixture.

* ``--gpus N`` under a launcher must equal WORLD_SIZE (an error, not a warning);
* without a launcher and N > 1, bench.py starts the N ranks itself and fails when a rank
  fails (here every rank fails: no GPU in this container), without hanging.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def test_gpus_must_match_world_size():
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=ROOT, capture_output=True, text=True,
                       timeout=120, env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"))
    assert p.returncode == 2 and "must match" in p.stderr
    assert p.stdout.strip() == ""


def test_self_launch_propagates_rank_failure():
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "1",
                        "--strong", "none"], cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env=_env(ADMM_DIST_BACKEND="gloo", CUDA_VISIBLE_DEVICES=""))
    assert p.returncode != 0
    assert "exited with" in p.stderr
    assert not any(l.startswith("{") for l in p.stdout.splitlines())


def test_cpu_baseline_reports_eq1_certificate():
    """The bench's CPU leg (oracle x-updates of node 0) carries rel_fro and the eq.(1)
    certificate of the oracle image; small case (32^2, 45 angles, 2 processes, 1 s)."""
    import numpy as np
    sys.path.insert(0, ROOT)
    import bench
    from oracle.geometry import Geometry, joseph_matrix, shepp_logan
    N, a = 32, 45
    A = joseph_matrix(Geometry(N, a))
    b = A @ shepp_logan(N, 2).ravel() + 0.005 * np.random.default_rng(0).standard_normal(A.shape[0])
    q = np.maximum(np.asarray(A.multiply(A).sum(axis=0)).ravel(), 1e-12)
    r = bench.cpu_baseline(N, a, b, q, np.zeros(N * N), procs=2, budget=1.0)
    assert r["kind"] == "port" and r["cores"] == 2 and r["value"] > 0
    assert abs(r["rel_fro"] - 1.0) < 1e-12  # x_gpu = 0 here
    c = r["eq1_gap"]
    assert c["m"] > 0 and c["dist_bound"] > 0 and c["obj_gap_bound"] >= c["eps"] >= 0
    assert c["dist_bound"] >= c["stationarity"] / c["m"]
    # eq.(1)'s objective at the oracle image and the gap bound relative to it
    assert c["objective"] > c["obj_gap_bound"] > 0
    assert abs(c["rel_obj_gap_bound"] - c["obj_gap_bound"] / c["objective"]) < 1e-15


def test_c4_graph_matches_committed_adjacency():
    """C4's Erdos-Renyi graph (32 nodes, p = 2 ln 32 / 32, seed 0, resampled
    until connected) is committed as a fixture; bench.make_graph must reproduce it exactly
    (a networkx change in the generator would silently change the C4 workload)."""
    import json
    import networkx as nx
    sys.path.insert(0, ROOT)
    from bench import make_graph
    with open(os.path.join(ROOT, "tests", "golden", "c4_er32_graph.json")) as f:
        fx = json.load(f)
    G = make_graph("er", 32)
    assert G.number_of_nodes() == fx["nodes"] == 32 and nx.is_connected(G)
    assert sorted([list(e) for e in G.edges()]) == fx["edges"]
    assert len(fx["edges"]) == 103


def test_roofline_traffic_lookup_finds_committed_kernels():
    """bench.py's roofline reads both projectors' PMC bytes per launch from the committed
    traffic files by their full template names (mirror mode at C3: 4-node real vectors,
    8-lane virtual ones)."""
    import json
    sys.path.insert(0, ROOT)
    import bench
    with open(os.path.join(ROOT, bench.TRAFFIC_FILES["C3"])) as fh:
        tr = json.load(fh)
    back = bench.back_kernel_traffic(tr, "float", 4, True)
    fwd = bench.fwd_kernel_traffic(tr, "float", 4, True)
    assert back is not None and fwd is not None
    # compulsory bytes of the C3 back launch (16 nodes, 512^2, 96 angles): sinogram + p + D + Hp
    # as float32 samples and r as float64 -- the PMC traffic exceeds it
    V, n, m = 16, 512 * 512, 96 * 512
    assert back > V * m * 4 + 3 * V * n * 4 + V * n * 8
    assert fwd > V * n * 4 + V * m * 4


def test_roofline_traffic_bound_to_kernel_sources(tmp_path, monkeypatch):
    """A PMC traffic file is used only if it records the hash of the kernel sources the
    library is built from; otherwise the line carries traffic null, the
    reason, and achieved on the compulsory bytes."""
    import json
    sys.path.insert(0, ROOT)
    import bench
    with open(os.path.join(ROOT, bench.TRAFFIC_FILES["C3"])) as fh:
        tr = json.load(fh)
    for sha, ok in ((bench.kernel_source_sha16(), True), ("0" * 16, False)):
        f = tmp_path / f"t_{ok}.json"
        f.write_text(json.dumps(dict(tr, kernel_source_sha16=sha)))
        monkeypatch.setitem(bench.TRAFFIC_FILES, "C3", str(f))
        bench.TRAFFIC_STALE.clear()
        got, _ = bench.pmc_traffic("C3")
        assert (got is not None) == ok
        assert ("C3" in bench.TRAFFIC_STALE) == (not ok)
    r = bench._roof("k", None, str(f), 0.05, 8e7, 1e9, stale=bench.TRAFFIC_STALE["C3"])
    assert r["traffic"] is None and r["achieved_basis"] == "compulsory" and "source hash" in r["traffic_source"]
    assert abs(r["frac"] - 8e7 / 0.05e-3 / 1e9 / bench.HBM_PEAK_GBS) < 1e-12


def test_committed_traffic_matches_kernel_sources():
    """The committed traffic files were measured on the kernels the sources build today."""
    sys.path.insert(0, ROOT)
    import bench
    for wl in ("C3", "weak8"):
        bench.TRAFFIC_STALE.clear()
        tr, f = bench.pmc_traffic(wl)
        assert tr is not None, bench.TRAFFIC_STALE
