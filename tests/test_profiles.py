"""The measured counters bench.py reports must belong to the kernel that ships.

bench.py takes HBM bytes and VALU utilisation from profiles/pmc.json only when an entry was
measured on the same kernel build (pyrenderer_amd.build.kernel_sha(): a hash of the device and
host sources and compile flags) and variant; otherwise its line carries null counters.  Round 2's
driver line lost them to an unprofiled edit.  This test fails as soon as a kernel-affecting edit
lands without a fresh profile of the headline workloads (tools/round_full.sh, tools/round_collect.sh).
"""
import csv
import json
import os
import re

import pytest

from conftest import ROOT

PMC = os.path.join(ROOT, "profiles", "pmc.json")
FINAL = os.path.join(ROOT, "profiles", "r06", "final")
# headline workloads: config 2 (bench.py default) on the LDS-resident pooled-shadow kernel, config 4
# on the global-scene kernel
KEYS = {"cornell_512x512x64spp_d8": ("prof_c2", 7), "cubes_512x512x64spp_d8": ("prof_c4", 3)}


@pytest.mark.parametrize("key", sorted(KEYS))
def test_pmc_entry_is_for_this_kernel_build(key):
    from pyrenderer_amd.build import kernel_sha
    e = json.load(open(PMC))[key]
    assert e["kernel_sha"] == kernel_sha(), (key, e["kernel_sha"], kernel_sha())
    assert e["variant"] == KEYS[key][1]
    assert e["hbm_bytes_per_launch"] > 0 and 0 < e["valu_issue_util"] <= 1 and 0 < e["valu_lane_util"] <= 1


@pytest.mark.parametrize("key", sorted(KEYS))
def test_rocprof_summary_agrees_with_the_bench_events(key):
    """The committed rocprofv3 kernel-trace summary and the bench line of the same profile run
    time the same kernel: its average duration (rocprof) and the HIP-event average (bench.py)
    agree within 5 %."""
    d = os.path.join(FINAL, KEYS[key][0])
    line = json.loads(open(os.path.join(d, "bench.json")).read().strip().splitlines()[-1])
    kname = line["roofline"]["kernel"]
    # the timed (non-STATS) instantiation; bench.py's counting pass runs the STATS one once
    rows = [r for r in csv.DictReader(open(os.path.join(d, "kernel_stats.csv")))
            if kname + "<" in r["Name"] and not re.search(r"trace_kernel(_pool)?<(\d+, )?true", r["Name"])]
    assert len(rows) == 1, [r["Name"] for r in rows]
    rocprof_ms = float(rows[0]["AverageNs"]) / 1e6
    assert abs(rocprof_ms - line["roofline"]["kernel_avg_ms"]) <= 0.05 * rocprof_ms, (rocprof_ms, line["roofline"])
    assert line["roofline"]["kernel_sha"] == json.load(open(PMC))[key]["kernel_sha"]


def test_no_roofline_fraction_above_one():
    """Every committed bench line of this round prices its work against a resource it can actually
    saturate: no `frac` field anywhere in the line exceeds 1 (round 3's `hbm_logical` priced LDS reads
    against the HBM peak and read 1.06)."""
    import glob

    def fracs(o, path=""):
        if isinstance(o, dict):
            for k, v in o.items():
                if k == "frac" and isinstance(v, (int, float)):
                    yield path + "/" + k, v
                yield from fracs(v, path + "/" + k)

    files = sorted(glob.glob(os.path.join(FINAL, "bench_all", "c*.json")))
    assert len(files) == 5
    for f in files:
        line = json.loads(open(f).read().strip().splitlines()[-1])
        bad = [(p, v) for p, v in fracs(line) if not 0 <= v <= 1]
        assert not bad, (f, bad)
