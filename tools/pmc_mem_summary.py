"""Summary of tools/pmc_mem.sh's passes for the trace kernel (median over its timed dispatches):
TA / TD busy fractions, L2 read requests and their mean latency, VMEM instruction level.

    python tools/pmc_mem_summary.py <outdir>
"""
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import med, per_dispatch  # noqa: E402


def main():
    d = sys.argv[1]
    r = {}
    for sub in ("ta", "tcp", "sq"):
        rows = per_dispatch(f"{d}/{sub}")
        for k in sorted({k for v in rows.values() for k in v}):
            r[f"{sub}.{k}"] = med(rows, k)
    # GRBM_GUI_ACTIVE comes summed over the 8 XCDs (8 x ~40 M cycles for an 18 ms dispatch at
    # ~2.25 GHz): per-XCD cycles = sum / 8; TA / TD / TCP have one instance per CU (256)
    n_xcd, n_cu = 8, 256
    g = (r.get("ta.GRBM_GUI_ACTIVE") or n_xcd) / n_xcd
    out = {
        "dispatch_ms": round(r["ta._ns"] / 1e6, 4),
        # TA / TD instances: one per CU
        "ta_busy": round(r["ta.TA_TA_BUSY_sum"] / (n_cu * g), 4),
        "ta_addr_stalled_by_tc": round(r["ta.TA_ADDR_STALLED_BY_TC_CYCLES_sum"] / (n_cu * g), 4),
        "td_busy": round(r["ta.TD_TD_BUSY_sum"] / (n_cu * g), 4),
        "td_tc_stall": round(r["ta.TD_TC_STALL_sum"] / (n_cu * g), 4),
        "tcp_pending_stall": round(r["tcp.TCP_PENDING_STALL_CYCLES_sum"] / (n_cu * r["tcp.GRBM_GUI_ACTIVE"] / n_xcd), 4),
        "l2_read_req_per_launch": r["tcp.TCP_TCC_READ_REQ_sum"],
        "l2_read_latency_cycles": round(r["tcp.TCP_TCC_READ_REQ_LATENCY_sum"] / max(r["tcp.TCP_TCC_READ_REQ_sum"], 1), 1),
        "l1_accesses_per_launch": r["tcp.TCP_TOTAL_CACHE_ACCESSES_sum"],
        "l1_accesses_per_cu_cycle": round(r["tcp.TCP_TOTAL_CACHE_ACCESSES_sum"] / (n_cu * r["tcp.GRBM_GUI_ACTIVE"] / n_xcd), 4),
        "l1_accesses_per_vmem_inst": round(r["tcp.TCP_TOTAL_CACHE_ACCESSES_sum"] / max(r["sq.SQ_INSTS_VMEM_RD"], 1), 2),
        "vmem_rd_insts": r["sq.SQ_INSTS_VMEM_RD"],
        "lds_insts": r["sq.SQ_INSTS_LDS"],
        # mean VMEM instructions in flight per wave: SQ_INST_LEVEL_VMEM accumulates the in-flight
        # count per cycle (quad-cycles, like SQ_WAVE_CYCLES)
        "vmem_in_flight_per_wave": round(r["sq.SQ_INST_LEVEL_VMEM"] / max(r["sq.SQ_WAVE_CYCLES"], 1), 3),
        "wait_inst_any_frac": round(r["sq.SQ_WAIT_INST_ANY"] / max(r["sq.SQ_WAVE_CYCLES"], 1), 4),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
