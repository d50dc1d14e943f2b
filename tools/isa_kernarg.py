"""ISA checks of the kernarg re-reads (prt_device.h kernarg()).

The LDS-scene kernels read their launch parameters through the kernarg segment pointer, which arrives
in s[0:1].  For that to be right, every kernel that re-reads must copy s[0:1] before anything writes
s0 or s1.  The point of the change is also that the production builds spill no SGPRs.

    python tools/isa_kernarg.py [listing.s ...]      (default: compile prt_trace_pool.hip)

Prints one line per trace kernel and exits non-zero on a violation.
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# a write to s0 / s1 (or a register tuple starting at s0) as the destination operand
_WRITE = re.compile(r"^(s_|v_readfirstlane|v_readlane|v_cmp)\S* (s0|s1|s\[0:\d+\])(,|$)")
_COPY = re.compile(r"^s_mov_b64 s\[\d+:\d+\], s\[0:1\]$")


def kernels(listing):
    """(name, instruction lines, metadata dict) per trace kernel in a hipcc -S listing."""
    s = open(listing).read()
    meta = {}
    for m in re.finditer(r"\.name:\s+(\S+)\n(.*?)(?=\n  - |\n\.\.\.|\Z)", s, re.S):
        fields = dict(re.findall(r"\.(\w+):\s+(\S+)", m.group(2)))
        meta[m.group(1)] = fields
    out = []
    for m in re.finditer(r"^(_Z\S*trace_kernel\S*):", s, re.M):
        name = m.group(1)
        j = s.index(".Lfunc_end", m.end())
        body = [ln.split(";")[0].strip() for ln in s[m.end():j].split("\n")]
        body = [ln for ln in body if ln and not ln.startswith(".") and not ln.endswith(":")]
        out.append((name, body, meta.get(name, {})))
    return out


def check(listing, reload_kernels=r"trace_kernel_pool"):
    """Violations: a re-reading kernel that writes s0/s1 before copying s[0:1], or (its production
    instantiations, no STATS) that spills SGPRs."""
    bad = []
    for name, body, meta in kernels(listing):
        if not re.search(reload_kernels, name):
            continue
        copies = [k for k, ln in enumerate(body) if _COPY.match(ln)]
        writes = [k for k, ln in enumerate(body) if _WRITE.match(ln)]
        first = copies[0] if copies else None
        early = [k for k in writes if first is None or k < first]
        spills = int(meta.get("sgpr_spill_count", 0))
        stats = "ILb1E" in name
        print(f"{name[-58:]}: kernarg copy at {first}, writes before {early[:3]}, SGPR spills {spills}")
        if first is None or early:
            bad.append(f"{name}: kernarg pointer not copied before s0/s1 are written")
        if not stats and spills:
            bad.append(f"{name}: {spills} SGPR spills")
    return bad


def compile_pool(out):
    from pyrenderer_amd import build as B
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    unit = "prt_trace_pool.hip"
    cmd = [hipcc] + B.FLAGS + B.UNIT_FLAGS.get(unit, []) + ["--cuda-device-only", "-S",
                                                          os.path.join(B.CSRC, unit), "-o", out]
    cmd = [c for c in cmd if c != "-fPIC"]
    subprocess.check_call(cmd, stderr=subprocess.DEVNULL)


def main():
    listings = sys.argv[1:]
    if not listings:
        tmp = os.path.join(tempfile.mkdtemp(), "pool.s")
        compile_pool(tmp)
        listings = [tmp]
    bad = []
    for ls in listings:
        bad += check(ls)
    for b in bad:
        print("FAIL", b)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
