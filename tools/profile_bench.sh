#!/bin/bash
# Bench + rocprofv3 kernel-trace summary + PMC passes (HBM bytes, VALU issue) for one config.
#   bash tools/profile_bench.sh <config> <outdir>     (on the GPU box, from the repo root)
# Then, here: python tools/pmc_summary.py --dir <outdir> --key <scene>_<W>x<H>x<spp>spp_d<depth>
set -e
CFG=${1:-2}
OUT=${2:-gpurun_out/prof_c$CFG}
mkdir -p $OUT
export TMPDIR=/tmp
# config 1 (0.06 ms per frame) runs bench_all.sh's 400 steps, so its launches hold the same 16 frames
ST=""; PST="--steps 10 --warmup 1"
[ $CFG = 1 ] && ST="--steps 400 --warmup 20" && PST="--steps 400 --warmup 20"
timeout -k 10 400 python3 bench.py --config $CFG $ST --single-frame-steps 0 > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o k --output-format csv -- python3 bench.py --config $CFG $ST --no-cpu-baseline --single-frame-steps 0 > $OUT/bench_under_rocprof.json 2> $OUT/rocprof_trace.err
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/fetch -o f --output-format csv -- python3 bench.py --config $CFG --no-cpu-baseline --single-frame-steps 0 $PST > /dev/null 2> $OUT/rocprof_fetch.err
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/write -o w --output-format csv -- python3 bench.py --config $CFG --no-cpu-baseline --single-frame-steps 0 $PST > /dev/null 2> $OUT/rocprof_write.err
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq -o s --output-format csv -- python3 bench.py --config $CFG --no-cpu-baseline --single-frame-steps 0 $PST > /dev/null 2> $OUT/rocprof_sq.err
echo done
