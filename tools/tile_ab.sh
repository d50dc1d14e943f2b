#!/bin/bash
# Tile-size A/B per config on one GPU: a wave's 64 work items cover one 64-pixel strip of a
# 64x64 tile, a 16x4 block of a 16x16 tile or a whole 8x8 tile (squarer = more coherent rays).
#   bash tools/tile_ab.sh <outdir> "<configs>" "<tiles>" [rounds]
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/tile_ab}; CONFIGS=${2:-"4 2 3"}; TILES=${3:-"64 16 8"}; ROUNDS=${4:-2}
mkdir -p $O
for c in $CONFIGS; do
  for r in $(seq 1 $ROUNDS); do
    for t in $TILES; do
      timeout -k 10 300 python3 bench.py --config $c --tile $t --no-cpu-baseline --numpy-seconds 0 \
        > $O/c${c}_t${t}_r${r}.json 2> $O/c${c}_t${t}_r${r}.err
      python3 -c "import json,sys; d=json.load(open('$O/c${c}_t${t}_r${r}.json')); print('c$c t$t r$r', round(d['value'],1), round(d['ms_per_step'],3), (d.get('l2_vs_cpu') or {}).get('pass'))"
    done
  done
done
