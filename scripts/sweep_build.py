"""Build tuning variants of the library into variants/ (gitignored .so; shipped by gpurun)."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, "distributed-inverse-problem-admm_amd")
from admm_hip.build import build  # noqa: E402

os.makedirs("variants", exist_ok=True)
variants = [tuple(map(int, v.split("x"))) for v in sys.argv[1:]]  # ROWSxSEG


def one(v):
    r, s = v
    return build(force=True, out=f"variants/lib_r{r}_s{s}.so", defines={"ADMM_FG_ROWS": r, "ADMM_FG_SEG": s})


with ThreadPoolExecutor(4) as ex:
    for p in ex.map(one, variants):
        print(p)
