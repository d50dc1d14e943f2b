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
SOURCES = ["prt_kernels.hip", "prt_capi.cpp", "prt_bvh.cpp", "prt_trace_pool.hip"]
# per-unit extra flags: the pooled-shadow kernel is register-allocated with LLVM's AMDGPU
# pressure trackers (4 instead of 39 spilled VGPRs at 7 waves/SIMD; prt_trace_pool.hip)
UNIT_FLAGS = {"prt_trace_pool.hip": ["-mllvm", "--amdgpu-use-amdgpu-trackers"]}
# the persistent trace kernel's instantiation sets: prt_trace_inst.hip compiled once
# per (traversal stack entries, stats) pair — the objects build in parallel
TRACE_INST = "prt_trace_inst.hip"
# stacks: 4 (the spill test's LDS part), 10 / 16 (LDS-resident scenes, the global scene's LDS
# part), 32 (deeper LDS-resident BVHs, PRT_SPILL_LDS=32)
TRACE_SETS = [(s, t) for s in (4, 10, 16, 32) for t in (0, 1)]
HEADERS = ["prt_kernels.h", "prt_internal.h", "prt_device.h"]
OBJ_DIR = os.path.join(LIB_DIR, "obj")
ARCH = os.environ.get("PRT_OFFLOAD_ARCH", "gfx950")

# -ffp-contract=off: f32 results must match oracle/prt_oracle.c bit for bit
# (DESIGN.md "Arithmetic contract"); division/sqrt stay correctly rounded
# (hipcc's default -fhip-fp32-correctly-rounded-divide-sqrt).
# -fno-slp-vectorize: packed-f32 SLP code pins constant pairs in VGPRs (spills at the
# occupancy targets) and is an anti-lever on CDNA4 (cdna_hip_programming.md, packed f32 VALU).
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-fno-slp-vectorize",
         f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function"]


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS + [TRACE_INST]] + [os.path.join(ROOT, "include", "prt.h"), __file__]
    return any(os.path.getmtime(p) > t for p in deps if os.path.exists(p))


def kernel_sha():
    """Short SHA-256 of the device/host sources and compile flags of libprt: keys the PMC
    summaries in profiles/pmc.json to the kernel build they were measured on (bench.py marks
    counter figures of another build as stale instead of reporting them)."""
    import hashlib
    h = hashlib.sha256()
    for f in sorted(SOURCES + HEADERS + [TRACE_INST]):
        h.update(f.encode())
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(FLAGS).encode())
    h.update(repr(sorted(UNIT_FLAGS.items())).encode())
    return h.hexdigest()[:16]


def _jobs():
    n = os.environ.get("MAX_JOBS") or os.cpu_count() or 4
    return max(1, min(int(n), 16))


def build(force=False, verbose=False, out=None, defs=()):
    """Build libprt.so (or, for A/B experiments, a copy at `out` compiled with extra -D `defs`)."""
    lib = out or LIB
    if out is None and not force and not _stale():
        return LIB
    obj_dir = OBJ_DIR if out is None else os.path.join("/tmp", "prt_ab_obj", os.path.basename(os.path.splitext(out)[0]))
    os.makedirs(obj_dir, exist_ok=True)
    os.makedirs(os.path.dirname(os.path.abspath(lib)), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    extra = [f"-D{d}" for d in defs]
    if out is not None:
        # A/B builds only: extra compiler flags (e.g. "-mllvm --amdgpu-use-amdgpu-trackers")
        extra += os.environ.get("PRT_AB_FLAGS", "").split()
    units = [(os.path.join(CSRC, f), os.path.join(obj_dir, os.path.splitext(f)[0] + ".o"), UNIT_FLAGS.get(f, []))
             for f in SOURCES]
    units += [(os.path.join(CSRC, TRACE_INST), os.path.join(obj_dir, f"prt_trace_{st}_{tt}.o"),
               [f"-DPRT_STACK={st}", f"-DPRT_STATS={tt}"]) for st, tt in TRACE_SETS]
    cmds = [[hipcc] + FLAGS + extra + d + ["-c", src, "-o", obj] for src, obj, d in units]
    if verbose:
        print(f"compiling {len(cmds)} units with {_jobs()} jobs", flush=True)
    from concurrent.futures import ThreadPoolExecutor
    # longest units first (the trace instantiation sets)
    order = sorted(range(len(cmds)), key=lambda i: TRACE_INST not in cmds[i][-3])
    with ThreadPoolExecutor(_jobs()) as ex:
        procs = list(ex.map(lambda i: subprocess.run(cmds[i], capture_output=True, text=True), order))
    for i, r in zip(order, procs):
        if r.returncode != 0:
            sys.stderr.write(" ".join(cmds[i]) + "\n" + r.stdout + r.stderr)
            raise subprocess.CalledProcessError(r.returncode, cmds[i])
        if verbose and (r.stderr or r.stdout).strip():
            print(r.stdout + r.stderr, flush=True)
    tmp = lib + ".tmp"
    link = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + [obj for _, obj, _ in units] + ["-ldl"]
    if verbose:
        print(" ".join(link), flush=True)
    subprocess.check_call(link)
    os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--out", help="A/B copy of the library (e.g. abtmp/libprt_x.so)")
    ap.add_argument("--define", "-D", action="append", default=[], help="extra preprocessor definition")
    a = ap.parse_args()
    print(build(force=a.force, verbose=True, out=a.out, defs=a.define))
