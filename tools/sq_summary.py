"""Summarise rocprofv3 SQ counter CSVs of the trace kernel (per dispatch mean).
    python tools/sq_summary.py gpurun_out/sq/a11 gpurun_out/sq/b11 [--iters N]
"""
import csv
import glob
import os
import re
import sys


def load(dirs, kernel="trace_kernel", exclude=r"trace_kernel(_pool)?<(\d+, )?true"):
    acc = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                n = r["Kernel_Name"]
                if kernel not in n or re.search(exclude, n):
                    continue
                acc.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
                acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in acc.items()}


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    c = load(args)
    for k in sorted(c):
        print(f"{k:28s} {c[k]:.4g}")
    if "SQ_WAVES" in c:
        w = c["SQ_WAVES"]
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_SMEM"):
            if k in c:
                print(f"{k} per wave: {c[k] / w:.4g}")
    if "SQ_ACTIVE_INST_VALU" in c and "GRBM_GUI_ACTIVE" in c:
        # ACTIVE_INST_* in quad-cycles; GRBM_GUI_ACTIVE summed over 8 XCDs; 4 SIMD x 32 CU per XCD
        simd_cycles = c["GRBM_GUI_ACTIVE"] / 8 * 1024
        print(f"VALU busy (issue cycles / SIMD cycles): {4 * c['SQ_ACTIVE_INST_VALU'] / simd_cycles:.3f}")
    if "SQ_THREAD_CYCLES_VALU" in c and "SQ_ACTIVE_INST_VALU" in c:
        print(f"VALU lane utilisation: {c['SQ_THREAD_CYCLES_VALU'] / (64 * c['SQ_ACTIVE_INST_VALU']):.3f}")
    if "SQ_LDS_BANK_CONFLICT" in c and "SQ_ACTIVE_INST_LDS" in c:
        print(f"LDS bank conflict / active LDS: {c['SQ_LDS_BANK_CONFLICT'] / c['SQ_ACTIVE_INST_LDS']:.3f}")
