#!/bin/bash
# Camera rays from the camera kernel (default) vs generated inside the trace kernel
# (bench.py --no-primary-kernel), interleaved rounds.   bash tools/primary_ab.sh <outdir> "<configs>" [rounds]
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/primary_ab}; CONFIGS=${2:-"2 4"}; ROUNDS=${3:-2}
mkdir -p $O
for c in $CONFIGS; do
  for r in $(seq 1 $ROUNDS); do
    for m in kernel inline; do
      F=""; [ $m = inline ] && F="--no-primary-kernel"
      timeout -k 10 300 python3 bench.py --config $c --steps 30 $F --no-cpu-baseline --numpy-seconds 0 \
        > $O/c${c}_${m}_r${r}.json 2> $O/c${c}_${m}_r${r}.err
      python3 -c "import json; d=json.load(open('$O/c${c}_${m}_r${r}.json')); print('c$c $m r$r', round(d['value'],1), round(d['ms_per_step'],3), d['roofline']['kernel_avg_ms'])"
    done
  done
done
