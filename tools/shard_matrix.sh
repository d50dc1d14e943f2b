#!/bin/bash
# Tile size x frames in flight for the multi-GPU bench's shards, on one GPU (tools/shard_sim.py):
#   bash tools/shard_matrix.sh <outdir> [config]
set -e
cd $GRAFT_REPO_ROOT
O=$1; C=${2:-2}
mkdir -p $O
for s in 1 2 3; do
  timeout -k 10 300 python3 tools/shard_sim.py --config $C --tiles 64,32,16 --schemes latin --worlds 2,8 --streams $s --steps 12 > $O/c${C}_s$s.jsonl 2> $O/c${C}_s$s.err
  tail -n 9 $O/c${C}_s$s.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('s$s', d['tile'], d['world'], max(d['wall_ms']) if isinstance(d['wall_ms'],list) else d['wall_ms'], d.get('eff_wall'))"
done
