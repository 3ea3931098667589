"""GPU: bench.py keeps the driver contract -- one JSON line on stdout with the metric,
the whole-job value, timing fields, roofline and (optionally) the CPU baseline and the
strong-scaling line (task contract)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, env=None):
    out = subprocess.run([sys.executable, "bench.py", *args], cwd=ROOT, capture_output=True, text=True,
                         timeout=540, check=True, env=env).stdout
    lines = [l for l in out.splitlines() if l.strip().startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_line_contract(cuda):
    b = _run("--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--strong", "none", "--proxy", "none")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in b, k
    assert b["n_gpus"] == 1 and b["steps"] == 3 and b["warmup"] == 1
    assert b["unit"] == "node-updates/s" and b["higher_is_better"] is True
    # one GPU: the headline is BASELINE configs[2] itself (C3: 16-node ring at 512^2), a fixed
    # config; the 8-nodes-per-GPU share of the N > 1 weak-scaling runs rides along as weak8
    assert b["config"]["nodes"] == 16 and b["config"]["baseline_config"] == 2 and b["scaling"] == "strong"
    assert "configs[2]" in b["config"]["workload"] and b["config"]["angles_per_node"] == 96
    assert b["weak8"]["nodes"] == 8 and b["weak8"]["value"] > 0 and b["strong"] == []
    # value = node-updates of the whole job / timed wall time
    assert abs(b["value"] - b["config"]["nodes"] * 1e3 / b["ms_per_step"]) <= 1e-6 * b["value"]
    r = b["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["bound"] in ("hbm", "mfma") and 0 < r["frac"] <= 1
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-9
    assert 0 < r["lds"]["frac"] <= 1
    # the dominant kernel is the projector with the longer in-solve launch; both are reported
    rf, rb = b["roofline_fwd"], b["roofline_back"]
    assert r["kernel"] == max((rf, rb), key=lambda x: x["avg_launch_ms"])["kernel"]
    assert rb["kernel"].startswith("k_back") and rf["kernel"].startswith("k_fwdg")
    for x in (rf, rb):
        assert 0 < x["frac"] <= 1 and 0 < x["lds"]["frac"] <= 1
        # PMC traffic only from a file measured on kernels of the current source hash
        if x["traffic"] is None:
            assert x["achieved_basis"] == "compulsory" and "source hash" in (x["traffic_source"] or "") or \
                "missing" in (x["traffic_source"] or ""), x
        else:
            assert x["achieved_basis"] == "pmc" and x["traffic"] > x["compulsory_bytes"]
    # the bound forward plan at 512^2 runs in one round (<= 2 blocks per CU)
    assert rf["fwd_plan"]["active"] and rf["fwd_plan"]["blocks"] <= 512, rf["fwd_plan"]
    assert "workload" in b["config"] and "model" not in b["config"]


def test_bench_launches_its_own_ranks(cuda):
    """``python bench.py --gpus 2`` with no launcher spawns the two ranks itself (gloo on
    this one-GPU box; the driver's nccl default is unchanged) and relays rank 0's line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["ADMM_DIST_BACKEND"] = "gloo"
    b = _run("--gpus", "2", "--steps", "2", "--warmup", "1", "--strong", "none", env=env)
    assert b["n_gpus"] == 2 and b["config"]["nodes"] == 16 and b["scaling"] == "weak"
    assert b["exchange_check"]["ok"] and b["exchange_check"]["halo_rows"] == 4


@pytest.mark.timeout(600)
def test_bench_eight_ranks_with_strong_c4(cuda):
    """The driver's N = 8 command shape (``bench.py --gpus 8``, default strong legs C3, C4) as
    a gloo rehearsal on this one GPU: 64-node ring over 8 self-launched ranks, then C3's
    16-node ring (2 nodes per rank) and C4's 32-node ER graph (all-gather exchange on every
    rank) over the same 8 ranks."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["ADMM_DIST_BACKEND"] = "gloo"
    b = _run("--gpus", "8", "--steps", "1", "--warmup", "1", "--strong-steps", "1", env=env)
    assert b["n_gpus"] == 8 and b["config"]["nodes"] == 64
    assert b["exchange_check"]["ok"] and b["exchange_check"]["mode"] == "p2p"
    assert [s["config"] for s in b["strong"]] == ["C3", "C4"]
    assert all(s["value"] > 0 and s["scaling"] == "strong" for s in b["strong"])


def test_bench_config_line(cuda):
    b = _run("--config", "C2", "--steps", "2", "--warmup", "1")
    assert b["scaling"] == "strong" and b["config"]["nodes"] == 8 and b["config"]["image"] == 256
    assert b["value"] > 0


def test_bench_as_rank_share(cuda):
    """``--config C4 --as-rank 0/8``: rank 0's share of C4 on 8 GPUs bound on this GPU --
    4 local nodes (one batch at node-interleave width 4), its real halo rows and stored
    edges of the 103-edge ER graph, its p2p halo exchange priced, not run."""
    b = _run("--config", "C4", "--as-rank", "0/8", "--steps", "2", "--warmup", "1")
    sh = b["share"]
    assert b["unit"] == "ms/step" and b["value"] == sh["ms_per_step"] > 0
    assert sh["local_nodes"] == 4 and sh["vb"] == 4 and sh["batches"] == 1 and sh["rank"] == 0
    assert sh["halo_rows"] > 0 and sh["stored_edges"] > 0
    assert sh["exchange"]["mode"] == "p2p"
    assert sh["exchange"]["bytes_received"] == sh["halo_rows"] * 1024 * 1024 * 8


@pytest.mark.long
@pytest.mark.timeout(600)
def test_bench_default_proxies(cuda):
    """The default one-GPU line's per-rank proxies: C3 on 2 ranks, C4 on 2 / 4 / 8 ranks, C5 on 8
    and the weak headline on 8, each with its measured one-GPU time, the share's time and the
    predicted speedup.  (ADMM_TEST_LONG:
    the driver's own default bench run produces this line every round.)"""
    b = _run("--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--strong-steps", "1", "--proxy-steps", "1")
    px = b["proxy_8gpu"]
    assert set(k for k in px if "@" in k) == {"C3@2", "C4@2", "C4@4", "C4@8", "C5@8", "weak8@8"}
    w = px["weak8@8"]  # the N = 8 weak headline: 64 nodes, 8 per rank
    assert w["nodes"] == 64 and w["shares"][0]["local_nodes"] == 8 and w["predicted_speedup"] > 0
    assert abs(w["predicted_value"] - 64e3 / w["predicted_ms_per_step"]) < 1e-6 * w["predicted_value"]
    assert [s["config"] for s in b["strong"]] == ["C4"]
    for k in ("C3@2", "C4@2", "C4@4", "C4@8"):
        p = px[k]
        assert p["T1_ms_per_step"] > 0 and p["predicted_speedup"] > 0 and p["per_node_cost_ratio"] > 0
        assert all(s["ms_per_step"] > 0 for s in p["shares"])
    assert px["C3@2"]["T1_ms_per_step"] == b["ms_per_step"]  # the headline is C3 on this GPU
    assert px["C4@8"]["shares"][0]["vb"] == 4 and px["C3@2"]["shares"][0]["exchange"]["mode"] == "p2p"
