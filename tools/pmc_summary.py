"""Per-launch PMC summary of the trace kernel for one bench configuration, merged into
profiles/pmc.json under the key bench.py matches (`<scene>_<W>x<H>x<spp>spp_d<depth>`).

Collect on the GPU box (one counter pass each; tools/profile_bench.sh does all of it):
    rocprofv3 --kernel-trace --pmc FETCH_SIZE -d OUT/fetch ... -- python3 bench.py ...
    rocprofv3 --kernel-trace --pmc WRITE_SIZE -d OUT/write ... -- python3 bench.py ...
    rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU \
        SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d OUT/sq ... -- python3 bench.py ...
Then:
    python tools/pmc_summary.py --dir OUT --key cornell_512x512x64spp_d8

The entry records the kernel build (`kernel_sha`, pyrenderer_amd.build.kernel_sha()) and the
trace-kernel variant the counters were measured on, read from OUT/bench.json (the bench line
of the same profile run); bench.py reports the counter figures only for that build and variant.

HBM bytes (MI355X_MICROARCH.md §HBM): FETCH_SIZE / WRITE_SIZE are KiB per dispatch summed over
XCDs; on gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads, so the stored
`hbm_bytes_per_launch` = 2 x FETCH + WRITE is an upper bound (the raw sum is kept too).
VALU: a wave64 VALU instruction occupies its SIMD-32 for 2 cycles, so
issue utilisation = 2 x SQ_INSTS_VALU / (SIMDs x cycles of the dispatch), with the shader
clock taken from SQ_WAVE_CYCLES (quad-cycles) / SQ_WAVES over the dispatch duration (the
persistent grid's waves live the whole launch); lane utilisation =
SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU).
"""
import argparse
import csv
import glob
import json
import os
import re
import statistics

EXCLUDE = r"trace_kernel(_pool)?<(\d+, )?true"   # the STATS (instrumented) instantiations


def per_dispatch(d, kernel="trace_kernel"):
    """{dispatch: {counter: value, '_ns': duration}} for the kernel's dispatches under d."""
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if kernel not in name or re.search(EXCLUDE, name):
                continue
            e = out.setdefault(r["Dispatch_Id"], {})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            e["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return out


def med(rows, key):
    v = [r[key] for r in rows.values() if key in r]
    return statistics.median(v) if v else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True, help="directory holding fetch/ write/ sq/ rocprofv3 outputs")
    ap.add_argument("--key", required=True)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "profiles", "pmc.json"))
    ap.add_argument("--simds", type=int, default=1024, help="256 CUs x 4 SIMDs")
    a = ap.parse_args()
    e = {}
    fk, wk = per_dispatch(os.path.join(a.dir, "fetch")), per_dispatch(os.path.join(a.dir, "write"))
    if fk and wk:
        f, w = med(fk, "FETCH_SIZE") * 1024.0, med(wk, "WRITE_SIZE") * 1024.0
        e.update({"fetch_bytes_raw": f, "write_bytes": w, "hbm_bytes_raw": f + w, "hbm_bytes_per_launch": 2.0 * f + w})
    sq = per_dispatch(os.path.join(a.dir, "sq"))
    if sq:
        waves, wcyc, ns = med(sq, "SQ_WAVES"), med(sq, "SQ_WAVE_CYCLES"), med(sq, "_ns")
        clock_ghz = (4.0 * wcyc / waves) / ns if waves and ns else None
        cycles = ns * clock_ghz
        e.update({"valu_insts": med(sq, "SQ_INSTS_VALU"), "dispatch_ms": ns / 1e6, "clock_ghz": round(clock_ghz, 3),
                  "valu_issue_util": round(2.0 * med(sq, "SQ_INSTS_VALU") / (a.simds * cycles), 4),
                  "valu_lane_util": round(med(sq, "SQ_THREAD_CYCLES_VALU") / (64.0 * med(sq, "SQ_ACTIVE_INST_VALU")), 4)})
    if not e:
        raise SystemExit("no matching dispatches")
    bl = os.path.join(a.dir, "bench.json")
    if not os.path.exists(bl):
        raise SystemExit(f"{bl} missing: the bench line of the profiled run names the kernel build")
    rl = json.loads(open(bl).read().strip().splitlines()[-1])["roofline"]
    e["kernel_sha"] = rl["kernel_sha"]
    e["variant"] = rl["variant"]["variant"]
    e["note"] = ("FETCH_SIZE doubled per the gfx950 correction (upper bound); VALU issue utilisation = "
                 "2 cycles per wave64 instruction on a SIMD-32 over SIMDs x dispatch cycles")
    db = json.load(open(a.out)) if os.path.exists(a.out) else {}
    db[a.key] = e
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(db, open(a.out, "w"), indent=1, sort_keys=True)
    print(json.dumps({a.key: e}))


if __name__ == "__main__":
    main()
