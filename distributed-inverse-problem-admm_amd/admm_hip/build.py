"""Build libadmm_tomo.so in-tree with hipcc for gfx950 (no JIT cache, no pip install)."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(_HERE)
CSRC = os.path.join(PKG, "csrc")
OUT = os.path.join(_HERE, "libadmm_tomo.so")
SOURCES = ["admm_tomo.hip", "masks.hip"]
DEPS = SOURCES + ["kernels.hpp"]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    hdr = os.path.join(os.path.dirname(PKG), "include", "admm_tomo.h")
    deps = [os.path.join(CSRC, d) for d in DEPS] + [hdr]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False, out: str | None = None,
          defines: dict | None = None) -> str:
    """Build the library (``out``/``defines``: tuning variants for sweeps, never the default)."""
    target = out or OUT
    if not force and out is None and not needs_build():
        return OUT
    arch = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"
    if arch != "gfx950":
        # the kernels are written for CDNA4: 160 KiB of LDS per workgroup (k_consensus_derived<128>
        # declares 128 KiB, the back projector's windows + DIAG tile ~80 KiB), v_permlane32/16_swap
        # and LDS-DMA widths of gfx950
        raise RuntimeError(f"libadmm_tomo targets gfx950 (MI355X) only; PYTORCH_ROCM_ARCH={arch!r}")
    tmp = target + ".tmp"
    dflags = [f"-D{k}={v}" for k, v in (defines or {}).items()]
    # -ffp-contract=off: no compiler-formed fmas.  Contraction is decided per template
    # instantiation, so with it the same expression could round differently for batch widths
    # VB = 1 and VB = 4 (measured: k_fwd_combine<float, 1, 1> fused Ax*L - b into one fma,
    # <float, 4, 1> did not), and a node's result would depend on how many nodes share its
    # batch -- i.e. on the GPU count and on the operator groups.  Every fma the kernels
    # rely on is written explicitly (fma(), v_pk_fma asm).
    cmd = [hipcc(), f"--offload-arch={arch}", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
           "-Wall", "-Wno-unused-function", *dflags, "-o", tmp] + [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, target)
    return target


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
