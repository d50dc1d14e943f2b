#!/bin/bash
# Vector-memory pipeline counters (TA / TD / TCP) and VMEM instruction levels for one config's trace
# launches: is a global-scene traversal bound by the address/data path or by latency?
#   bash tools/pmc_mem.sh <config> <outdir>      (GPU box, repo root)
set -e
CFG=${1:-4}
OUT=${2:-gpurun_out/pmc_mem_c$CFG}
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --config $CFG --no-cpu-baseline --steps 2 --warmup 1 --frames-per-launch 1"
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE -d $OUT/ta -o t --output-format csv -- $B > /dev/null 2> $OUT/ta.err
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE -d $OUT/tcp -o c --output-format csv -- $B > /dev/null 2> $OUT/tcp.err
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq -o s --output-format csv -- $B > /dev/null 2> $OUT/sq.err
echo done
