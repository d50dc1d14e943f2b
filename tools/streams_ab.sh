#!/bin/bash
# Frames in flight at N = 1 (bench.py --streams): wall time per step and the in-bench
# trace-kernel event average, interleaved rounds.
#   bash tools/streams_ab.sh <outdir> "<configs>" "<streams>" [rounds]
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/streams_ab}; CONFIGS=${2:-"2 4"}; STREAMS=${3:-"1 2 3"}; ROUNDS=${4:-2}
mkdir -p $O
for c in $CONFIGS; do
  for r in $(seq 1 $ROUNDS); do
    for s in $STREAMS; do
      timeout -k 10 300 python3 bench.py --config $c --streams $s ${STEPS_ARGS:---steps 30} --no-cpu-baseline --numpy-seconds 0 \
        > $O/c${c}_s${s}_r${r}.json 2> $O/c${c}_s${s}_r${r}.err
      python3 -c "import json; d=json.load(open('$O/c${c}_s${s}_r${r}.json')); print('c$c s$s r$r', round(d['value'],1), round(d['ms_per_step'],3), d['roofline']['kernel_avg_ms'])"
    done
  done
done
