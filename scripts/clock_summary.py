"""Effective shader clock per kernel from a GRBM_GUI_ACTIVE pass (scripts/pmc.sh with
PASSFILE=scripts/passes_clock.txt): GRBM_GUI_ACTIVE / 8 XCDs / the dispatch's duration.
usage: python scripts/clock_summary.py DIR [kernel-substring ...]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
pats = sys.argv[2:] or ["k_fwdg<float, 8", "k_back_mirror_2<float, 8, 4>", "k_back_mirror<float, 8, 4, 3>", "k_cg_update", "k_tv_update"]
f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True) + glob.glob(f"{d}/*counter_collection.csv")
acc = collections.defaultdict(lambda: [0, 0.0, 0.0])
for r in csv.DictReader(open(f[0])):
    if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
        continue
    for p in pats:
        if p in r["Kernel_Name"]:
            a = acc[p]
            a[0] += 1
            a[1] += float(r["Counter_Value"])
            a[2] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
for p, (n, g, t) in acc.items():
    print(f"{p:40s} n={n:4d}  {t / n * 1e6:8.2f} us  GRBM/8/t = {g / 8 / t / 1e9:6.3f} GHz")
