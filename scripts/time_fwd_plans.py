"""Forward-projector plans side by side (admm_fwd_plan_info + event-timed k_fwdg launches).

For each image size (env SIZES, default "512:float32,1024:float32,2048:float64") and each
plan the geometry has (0: 64-ray chunks, 1: aligned per (segment, angle), 2: aligned per
(segment, chunk); 3-5: the same with rays clipped to each segment), binds an 8-node batch
with ADMM_FWD_PLAN forcing the plan and prints the planner's groups / blocks / staged pixels with the average tap-launch time back to back and
in-solve (one x-update's 50 CG-step forwards), one JSON line per (size, plan)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "distributed-inverse-problem-admm_amd"), ROOT]
import networkx as nx  # noqa: E402
import torch  # noqa: E402

from admm_hip.data import make_precisions, make_sinograms, shepp_logan  # noqa: E402
from admm_hip.plan import make_plan  # noqa: E402
from admm_hip.solver import NodeBatch, make_operators  # noqa: E402

V = int(os.environ.get("V", 8))
for item in os.environ.get("SIZES", "512:float32,1024:float32,2048:float64").split(","):
    n, dt = item.split(":")
    N = int(n)
    ops = make_operators(N, V, angles_total=96 * V, dtype=dt, device=0)
    plan = make_plan(nx.cycle_graph(V), V, 1, 0)
    ph = shepp_logan(N)
    sinos = dict(zip(plan.local_nodes, make_sinograms(ops, ph, 0.005, seed=1000)))
    Wi, Q = make_precisions(ops)
    for pl in range(6):
        os.environ["ADMM_FWD_PLAN"] = str(pl)
        nb = NodeBatch(ops[0].geom, dt, plan, sinos, Q, 2.0, 0.02, 0.2, 10, 5, "iso", ph, 0, keep_x=True)
        info = {p["plan"]: p for p in nb.fwd_plans()}
        if pl not in info:
            print(json.dumps({"N": N, "dtype": dt, "plan": pl, "available": False}), flush=True)
            del nb
            continue
        nb.node_update()
        torch.cuda.synchronize()
        b2b = [round(nb.time_forward(10 if N >= 2048 else 50) * 1e3, 2) for _ in range(2)]
        ins = round(nb.time_forward(in_solve=True) * 1e3, 2)
        print(json.dumps({"N": N, "dtype": dt, "plan": pl, **info[pl], "fwd_us_b2b": b2b,
                          "fwd_us_in_solve": ins}), flush=True)
        del nb
        torch.cuda.empty_cache()
    os.environ.pop("ADMM_FWD_PLAN", None)
