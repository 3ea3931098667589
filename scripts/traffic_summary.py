"""Per-launch and per-step HBM traffic from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
(scripts/pmc.sh runs bench.py with ADMM_BENCH_MARKERS=1: one k_tv_grad launch before and
one after the timed steps).  MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads,
so it is doubled (the projector staging, CG and TV kernels all read with 16-B or wider
vectors or 8-B lanes; the doubling is exact for the former and an upper bound for the
latter).  Both counters count Infinity-Cache (MALL) hits as memory traffic.

Per-kernel figures are averages over the launches inside the timed window; per_step is
the window's total divided by the number of timed steps.

usage: python scripts/traffic_summary.py <tag> <steps> <out.json>
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import KERNEL_SOURCES, kernel_source_sha16  # noqa: E402  (the hash bench.py checks)

tag, steps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
MARK = "k_tv_grad"


def window(rows, counter):
    """{dispatch: (kernel, value)} of one counter, restricted to the marked window."""
    d = {}
    for r in rows:
        if r["Counter_Name"] != counter:
            continue
        k = int(r["Dispatch_Id"])
        name, v = d.get(k, (r["Kernel_Name"], 0.0))
        d[k] = (name, v + float(r["Counter_Value"]))  # per-XCD/instance rows summed
    ids = sorted(d)
    marks = [k for k in ids if MARK in d[k][0]]
    if len(marks) < 2:
        raise SystemExit(f"{counter}: expected 2 marker launches, found {len(marks)}")
    lo, hi = marks[-2], marks[-1]
    return {k: d[k] for k in ids if lo < k < hi}


per = {}
for f in sorted(glob.glob(f"gpurun_out/{tag}_*/**/*counter_collection.csv", recursive=True)):
    rows = list(csv.DictReader(open(f)))
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        if any(r["Counter_Name"] == counter for r in rows):
            per[counter] = window(rows, counter)
if set(per) != {"FETCH_SIZE", "WRITE_SIZE"}:
    raise SystemExit(f"missing passes: have {sorted(per)}")
acc = collections.defaultdict(lambda: {"fetch": [], "write": []})
for key, which in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
    for _, (name, v) in per[key].items():
        acc[name.split("(")[0].replace("void ", "")][which].append(v * 1024.0)
res = {}
tot_f = tot_w = 0.0
for k, v in acc.items():
    nf, nw = len(v["fetch"]), len(v["write"])
    if nf == 0 or nw == 0 or nf != nw:
        raise SystemExit(f"{k}: launch counts differ between passes ({nf} vs {nw})")
    fetch, write = sum(v["fetch"]) / nf, sum(v["write"]) / nw
    tot_f += sum(v["fetch"])
    tot_w += sum(v["write"])
    res[k] = {"fetch_size_bytes": fetch, "write_size_bytes": write,
              "hbm_bytes_per_launch": 2.0 * fetch + write,
              "launches_per_step": nf / steps}
json.dump({"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), tag {tag}, "
                     f"launches between the bench's two marker kernels ({steps} timed steps)",
           "correction": "hbm = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), MI355X_MICROARCH.md HBM",
           "kernel_source_sha16": kernel_source_sha16(), "kernel_sources": list(KERNEL_SOURCES),
           "per_step": {"hbm_bytes": (2.0 * tot_f + tot_w) / steps, "fetch_size_bytes": tot_f / steps,
                        "write_size_bytes": tot_w / steps, "steps": steps},
           "kernels": res}, open(out, "w"), indent=1, sort_keys=True)
for k, r in sorted(res.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["launches_per_step"]):
    print(f"{r['hbm_bytes_per_launch']/1e6:10.2f} MB x {r['launches_per_step']:5.1f}/step  {k}")
print(f"per step: {(2.0 * tot_f + tot_w) / steps / 1e6:.1f} MB")
