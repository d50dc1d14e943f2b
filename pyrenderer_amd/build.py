"""Build libprt.so in-tree (pyrenderer_amd/lib/) with hipcc for gfx950.

The library travels to the GPU box inside the repo snapshot; nothing is
installed into site-packages.  `python -m pyrenderer_amd.build` or
`__graft_entry__.build()` runs this.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB_DIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIB_DIR, "libprt.so")
SOURCES = ["prt_kernels.hip", "prt_capi.cpp", "prt_bvh.cpp"]
HEADERS = ["prt_kernels.h", "prt_internal.h"]
ARCH = os.environ.get("PRT_OFFLOAD_ARCH", "gfx950")

# -ffp-contract=off: f32 results must match oracle/prt_oracle.c bit for bit
# (DESIGN.md "Arithmetic contract"); division/sqrt stay correctly rounded
# (hipcc's default -fhip-fp32-correctly-rounded-divide-sqrt).
# -fno-slp-vectorize: packed-f32 SLP code pins constant pairs in VGPRs (spills at the
# occupancy targets) and is an anti-lever on CDNA4 (cdna_hip_programming.md, packed f32 VALU).
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math", "-fno-slp-vectorize",
         f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function"]


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(ROOT, "include", "prt.h"), __file__]
    return any(os.path.getmtime(p) > t for p in deps if os.path.exists(p))


def build(force=False, verbose=False):
    if not force and not _stale():
        return LIB
    os.makedirs(LIB_DIR, exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    tmp = LIB + ".tmp"
    cmd = [hipcc] + FLAGS + ["-o", tmp] + [os.path.join(CSRC, f) for f in SOURCES]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
