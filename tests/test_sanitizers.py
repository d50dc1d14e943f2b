"""Host sanitizer builds: the host C++ of libprt's BVH pipeline
(pyrenderer_amd/csrc/prt_bvh.cpp — SAH binning, spatial splits with Sutherland-Hodgman clipping in
double, reference unsplitting, treelet restructuring over 127 subsets, the BVH4 collapse and the
quantiser) and the C oracle (oracle/prt_oracle.c) compiled with AddressSanitizer + UndefinedBehavior-
Sanitizer (float-to-int overflow included), every finding fatal (tools/sanitize/Makefile).  The
reference's nearest equivalent is its debug mode, ti.init(debug=True) (/root/reference/debug/run.py:7).

The quick part runs here: the BVH driver (tools/sanitize/bvh_check.cpp, which also checks every tree
structurally: leaves, nesting, cover of every triangle, BVH4 and quantised boxes, stack bound) over
random soups under all four PRT_SBVH / PRT_TREELET settings, degenerate inputs and the Cornell box,
and the fast part of the oracle's golden suite in a python process with the sanitizer runtime
preloaded.  `make -C tools/sanitize check` adds the config-4 sized build (1,000,044 triangles) and the
whole golden suite (logs: profiles/r06/sanitize/)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import CORNELL_JSON, ROOT

SAN = os.path.join(ROOT, "tools", "sanitize")
OUT = os.path.join(ROOT, "build", "sanitize")


@pytest.fixture(scope="module")
def built():
    subprocess.run(["make", "-s", "-C", SAN, "all"], check=True, capture_output=True, timeout=600)
    return OUT


def _check(built, args, **env):
    e = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1", **env)
    r = subprocess.run([os.path.join(built, "bvh_check")] + [str(a) for a in args], env=e, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("sbvh,treelet", [("0", "0"), ("1", "0"), ("0", "3"), ("1", "3")])
def test_bvh_pipeline_clean_under_asan_ubsan(built, sbvh, treelet):
    small = _check(built, ["--random", 3000, 3], PRT_SBVH=sbvh, PRT_TREELET=treelet)
    # >= 2^14 triangles: the large-scene build (64 bins, 128 x clipping threshold, treelets by default)
    large = _check(built, ["--random", 20000, 7, 8], PRT_SBVH=sbvh, PRT_TREELET=treelet)
    for rep in (small, large):
        assert rep["failures"] == 0 and rep["references"] >= rep["triangles"]
        assert (rep["spatial_splits"] > 0) == (sbvh == "1")


def test_bvh_degenerate_and_cornell_inputs_under_asan_ubsan(built, tmp_path):
    for n in (0, 1, 2, 9):
        assert _check(built, ["--random", n, 5])["triangles"] == n
    same = tmp_path / "same.f32"
    np.tile(np.array([[0, 0, 0, 1, 0, 0, 0, 1, 0]], np.float32), (50, 1)).tofile(same)
    assert _check(built, [same, 4])["references"] == 50
    from pyrenderer_amd.flatten import flatten_scene
    from pyrenderer_amd.io_utils.read_tungsten import read_file
    scene, _ = read_file(CORNELL_JSON)
    corn = tmp_path / "cornell.f32"
    flatten_scene(scene).tri_v.astype(np.float32).tofile(corn)
    rep = _check(built, [corn])
    assert rep["triangles"] == 36 and rep["spatial_splits"] == 0


def test_oracle_golden_kats_under_asan_ubsan(built):
    """The oracle's known-answer tests and both-backend checks against the sanitized build, in a python
    process with the sanitizer runtimes preloaded (the long scripted-replay tests run in `make check`)."""
    cc = os.environ.get("CC", "gcc")
    pre = ":".join(subprocess.run([cc, f"-print-file-name={lib}"], capture_output=True, text=True).stdout.strip()
                   for lib in ("libasan.so", "libubsan.so"))
    lib = os.path.join(built, "libprt_oracle.so")
    env = dict(os.environ, LD_PRELOAD=pre, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", PRT_ORACLE_LIB=lib)
    # the sanitized library is the one the oracle loads
    probe = subprocess.run([sys.executable, "-c", "from oracle import oracle as O; O.lib(); "
                            "print(any(l.rstrip().endswith('build/sanitize/libprt_oracle.so') "
                            "for l in open('/proc/self/maps')))"], cwd=ROOT, env=env, capture_output=True,
                           text=True, timeout=120)
    assert probe.returncode == 0 and probe.stdout.strip() == "True", probe.stdout + probe.stderr[-2000:]
    r = subprocess.run([sys.executable, "-m", "pytest", "tests/test_oracle_golden.py", "-q", "-p", "no:cacheprovider",
                        "-k", "not scripted and not moller and not mis_direct and not sphere_and_bsdf"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert " passed" in r.stdout and "AddressSanitizer" not in r.stderr
