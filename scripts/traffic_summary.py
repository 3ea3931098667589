"""Per-launch HBM traffic per kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
(scripts/pmc.sh).  MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads, so it is
doubled (the projector staging, CG and TV kernels all read with 16-B or wider vectors
or 8-B lanes; the doubling is exact for the former and an upper bound for the latter).

usage: python scripts/traffic_summary.py <tag> <out.json>
"""
import collections
import csv
import glob
import json
import sys

tag, out = sys.argv[1], sys.argv[2]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"gpurun_out/{tag}_*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {}
for k, v in vals.items():
    if "FETCH_SIZE" not in v or "WRITE_SIZE" not in v:
        continue
    fetch = sum(v["FETCH_SIZE"]) / len(v["FETCH_SIZE"]) * 1024.0
    write = sum(v["WRITE_SIZE"]) / len(v["WRITE_SIZE"]) * 1024.0
    short = k.split("(")[0].replace("void ", "")
    res[short] = {"fetch_size_bytes": fetch, "write_size_bytes": write,
                  "hbm_bytes_per_launch": 2.0 * fetch + write,
                  "launches_sampled": len(v["FETCH_SIZE"])}
json.dump({"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), tag {tag}",
           "correction": "hbm = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), MI355X_MICROARCH.md HBM",
           "kernels": res}, open(out, "w"), indent=1, sort_keys=True)
for k, r in sorted(res.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"]):
    print(f"{r['hbm_bytes_per_launch']/1e6:10.2f} MB  {k}")
