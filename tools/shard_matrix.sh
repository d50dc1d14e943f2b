#!/bin/bash
# Tile size x frames in flight x kernel variant for the multi-GPU bench's shards, on one GPU
# (tools/shard_sim.py; efficiencies against this process's own one-GPU frame):
#   STREAMS="1 2 3" TILES=64,32,16 WORLDS=2,8 VARIANTS=0 bash tools/shard_matrix.sh <outdir> [config]
set -e
cd $GRAFT_REPO_ROOT
O=$1; C=${2:-2}
mkdir -p $O
for v in ${VARIANTS:-0}; do for s in ${STREAMS:-1 2 3}; do
  f=$O/c${C}_v${v}_s$s.jsonl
  timeout -k 10 300 python3 tools/shard_sim.py --config $C --tiles ${TILES:-64,32,16} --schemes latin --worlds ${WORLDS:-2,8} \
    --streams $s --steps 12 --variant $v > $f 2> $O/err.log
  python3 -c "
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    w = max(d['wall_ms']) if isinstance(d['wall_ms'], list) else d['wall_ms']
    print('v$v s$s tile', d['tile'], 'world', d['world'], 'slowest rank ms', w, 'eff', d.get('eff_wall'))" $f
done; done
