#!/bin/bash
# One bench line per BASELINE config on one GPU.  bash tools/bench_all.sh <outdir>
set -e
OUT=${1:-gpurun_out/bench_all}
mkdir -p $OUT
for c in 1 2 3 4 5; do
  timeout -k 10 400 python3 bench.py --config $c > $OUT/c$c.json 2> $OUT/c$c.err
  tail -c 400 $OUT/c$c.json
done
