#!/bin/bash
# One bench line per BASELINE config on one GPU.  bash tools/bench_all.sh <outdir>
set -e
OUT=${1:-gpurun_out/bench_all}
mkdir -p $OUT
for c in 1 2 3 4 5; do
  # config 1 is 0.06 ms per step: 400 steps give a timed region of ~25 ms instead of 0.6 ms
  STEPS=""; [ $c = 1 ] && STEPS="--steps 400 --warmup 20"
  timeout -k 10 400 python3 bench.py --config $c $STEPS > $OUT/c$c.json 2> $OUT/c$c.err
  tail -c 400 $OUT/c$c.json
done
