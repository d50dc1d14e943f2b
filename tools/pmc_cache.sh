#!/bin/bash
# L2 / HBM / issue counters of the trace kernel for one config and variant.
#   CFG=4 VAR=9 bash tools/pmc_cache.sh gpurun_out/cache_c4
set -e
OUT=${1:-gpurun_out/cache}
CFG=${CFG:-4}
VAR=${VAR:-0}
mkdir -p $OUT
export TMPDIR=/tmp
run() { timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$1 -o p --output-format csv -- python3 tools/one_render.py --config $CFG --variant $VAR --reps 1 > $OUT/$1.log 2>&1; }
run TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum
run FETCH_SIZE
run SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE
echo done
