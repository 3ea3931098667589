"""VGPR / SGPR / scratch / LDS of each kernel from a hipcc -save-temps .s (amdhsa metadata).
usage: python scripts/kernel_resources.py file.s [name-substring ...]"""
import re
import subprocess
import sys

txt = open(sys.argv[1]).read()
meta = txt[txt.index("amdhsa.kernels:"):]
want = sys.argv[2:]
for blk in re.split(r"\n  - ", meta)[1:]:
    f = dict(re.findall(r"^\s+\.([a-z_]+):\s+(\S+)", blk, re.M))
    name = f.get("name", "?")
    if want and not any(w in name for w in want):
        continue
    dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    print(f"{dem[:70]:70s} vgpr {f.get('vgpr_count'):>4} sgpr {f.get('sgpr_count'):>4} "
          f"spill {f.get('vgpr_spill_count', '0'):>3} scratch {f.get('private_segment_fixed_size'):>4} "
          f"lds {f.get('group_segment_fixed_size'):>6}")
