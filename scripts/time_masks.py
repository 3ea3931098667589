"""Setup timing of the per-pixel mask builder: HIP kernel vs the
oracle's per-pixel numpy/networkx loop (the reference's algorithm) on a pixel sample."""
import json
import sys
import time

import numpy as np
import torch

sys.path[:0] = ["distributed-inverse-problem-admm_amd", "."]
from admm_hip.masks import chain_orders, pixel_masks  # noqa: E402
from oracle import masks as om  # noqa: E402

out = []
for N, V in ((512, 16), (1024, 32)):
    n = N * N
    rng = np.random.default_rng(0)
    W = [np.exp(0.5 * rng.standard_normal(n)) for _ in range(V)]
    for strat in ("knn", "mst", "chain"):
        pixel_masks(W, strat, k=2)  # warm (module load, kernel)
        torch.cuda.synchronize()
        t = time.perf_counter()
        keep = pixel_masks(W, strat, k=2)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        t = time.perf_counter()
        chain_orders(V, n) if strat == "chain" else None
        dt_orders = time.perf_counter() - t if strat == "chain" else 0.0
        S = 300  # oracle pixel sample
        Ws = [w[:S] for w in W]
        _, q = om.precisions(Ws)
        t = time.perf_counter()
        om.build_all_masks(q, V, S, strategy=strat, k=2)
        per_px = (time.perf_counter() - t) / S
        rec = dict(N=N, V=V, strategy=strat, gpu_s=round(dt, 4), chain_orders_host_s=round(dt_orders, 4),
                   oracle_s_per_pixel=per_px, oracle_extrapolated_s=round(per_px * n, 1),
                   keep_bytes=int(keep.numel()))
        print(json.dumps(rec), flush=True)
        out.append(rec)
        del keep
        torch.cuda.empty_cache()
json.dump(out, open("gpurun_out/time_masks.json", "w"), indent=1)
