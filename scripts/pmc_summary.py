"""Summarise rocprofv3 --pmc CSVs per kernel (mean over dispatches)."""
import collections
import csv
import glob
import sys

tag = sys.argv[1]
keys = sys.argv[2:] or ["k_fwdg<float, 8>", "k_fwd<float, 8, 0", "k_back<float, 8, 3", "k_cg_update<float, 8", "k_tv_update<float, 8, false"]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(f"gpurun_out/{tag}_*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    for key in keys:
        if key in k:
            print(f"== {k[:70]}")
            for c, xs in sorted(v.items()):
                print(f"   {c:28s} {sum(xs)/len(xs):14.6g}  (n={len(xs)})")
