"""Build tuning variants of the library into variants/ (gitignored .so; shipped by gpurun)."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, "distributed-inverse-problem-admm_amd")
from admm_hip.build import build  # noqa: E402

os.makedirs("variants", exist_ok=True)
# each argument: NAME:MACRO=VAL,MACRO=VAL   e.g.  seg16:ADMM_FG_SEG=16
variants = []
for a in sys.argv[1:]:
    name, _, defs = a.partition(":")
    variants.append((name, dict(kv.split("=") for kv in defs.split(",") if kv)))


def one(v):
    name, defs = v
    return build(force=True, out=f"variants/lib_{name}.so", defines=defs)


with ThreadPoolExecutor(4) as ex:
    for p in ex.map(one, variants):
        print(p)
