#!/bin/bash
# VGPR / spill counts of the trace-kernel variants for one instantiation set (device ISA only)
#   bash tools/isa_regs.sh <stack> [-DFOO ...]
ST=$1; shift
OUT=/tmp/isa_regs_$$.s
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fno-slp-vectorize --offload-arch=gfx950 \
  --cuda-device-only -S -DPRT_STACK=$ST -DPRT_STATS=0 "$@" pyrenderer_amd/csrc/prt_trace_inst.hip -o $OUT 2>/dev/null
awk '/\.name:.*trace_kernel/{n=$2} /\.vgpr_count:/{v=$2} /\.vgpr_spill_count:/{print n, "vgpr", v, "spill", $2}' $OUT | sed 's/_ZN3prt12_GLOBAL__N_112trace_kernelI//'
rm -f $OUT
