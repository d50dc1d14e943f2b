#!/bin/bash
# Per-launch buffer budget (PRT_CHUNK_BYTES: per-sample radiance + primary rays per trace launch)
# at configs 3 and 5: fewer, larger launches = fewer launch tails per frame.
#   bash tools/chunk_ab.sh <outdir> "<configs>" "<GiB values>" [rounds]
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/chunk_ab}; CONFIGS=${2:-"3 5"}; GIBS=${3:-"4 16 64"}; ROUNDS=${4:-2}
mkdir -p $O
for c in $CONFIGS; do
  STEPS="--steps 10"; [ $c = 5 ] && STEPS="--steps 4 --warmup 1"
  for r in $(seq 1 $ROUNDS); do
    for g in $GIBS; do
      PRT_CHUNK_BYTES=$((g << 30)) timeout -k 10 300 python3 bench.py --config $c $STEPS --no-cpu-baseline \
        --numpy-seconds 0 > $O/c${c}_g${g}_r${r}.json 2> $O/c${c}_g${g}_r${r}.err
      python3 -c "import json; d=json.load(open('$O/c${c}_g${g}_r${r}.json')); rf=d['roofline']; print('c$c ${g}GiB r$r', round(d['value'],1), round(d['ms_per_step'],3), rf['kernel_avg_ms'], rf['launches_per_step'])"
    done
  done
done
