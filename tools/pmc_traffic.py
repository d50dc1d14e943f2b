"""HBM traffic of the trace kernel from rocprofv3 PMC passes.

Collect (separate passes: FETCH_SIZE and WRITE_SIZE do not fit one TCC pass):
    rocprofv3 --kernel-trace --pmc FETCH_SIZE -d OUT/fetch -o f --output-format csv -- python bench.py ...
    rocprofv3 --kernel-trace --pmc WRITE_SIZE -d OUT/write -o w --output-format csv -- python bench.py ...
Then:
    python tools/pmc_traffic.py --fetch OUT/fetch --write OUT/write --config 512x512x64spp_d8 --out profiles/traffic.json

FETCH_SIZE / WRITE_SIZE are KiB per dispatch (summed over XCDs).  MI355X_MICROARCH.md §HBM:
on gfx950 FETCH_SIZE counts exactly half the bytes of wide coalesced streaming reads
(128-B requests tallied as 64 B), WRITE_SIZE is exact for 16-B streaming stores; other widths
are uncalibrated.  Both the raw sum and the read-corrected sum (FETCH x 2 + WRITE) are stored;
`hbm_bytes_per_launch` is the corrected (upper) figure.
"""
import argparse
import csv
import re
import glob
import json
import os
import statistics


def per_dispatch(d, counter, kernel_substr, exclude_substr):
    rows = []
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        rows += list(csv.DictReader(open(f)))
    acc = {}
    for r in rows:
        name = r["Kernel_Name"]
        if kernel_substr not in name or (exclude_substr and re.search(exclude_substr, name)):
            continue
        if r["Counter_Name"] != counter:
            continue
        acc[r["Dispatch_Id"]] = acc.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(acc.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--config", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--kernel", default="trace_kernel")
    ap.add_argument("--exclude", default=r"trace_kernel<\d+, true", help="regex: skip the STATS (instrumented) instantiation")
    a = ap.parse_args()
    fk = per_dispatch(a.fetch, "FETCH_SIZE", a.kernel, a.exclude)
    wk = per_dispatch(a.write, "WRITE_SIZE", a.kernel, a.exclude)
    if not fk or not wk:
        raise SystemExit("no matching dispatches")
    f = statistics.median(fk) * 1024.0
    w = statistics.median(wk) * 1024.0
    out = {"config": a.config, "kernel": a.kernel, "fetch_bytes_raw": f, "write_bytes": w,
           "hbm_bytes_raw": f + w, "hbm_bytes_per_launch": 2.0 * f + w,
           "dispatches": {"fetch": len(fk), "write": len(wk)},
           "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md gfx950 correction (upper bound for non-streaming reads)"}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
