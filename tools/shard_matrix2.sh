set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03/shardm2; mkdir -p $O
for v in 0 7; do for s in 3 4 6; do
  timeout -k 10 300 python3 tools/shard_sim.py --config 2 --tiles 32,16 --schemes latin --worlds 4,8 --streams $s --steps 12 --variant $v > $O/c2_v${v}_s$s.jsonl 2> $O/err.log
  python3 -c "
import json,sys
for l in open('$O/c2_v${v}_s$s.jsonl'):
    d=json.loads(l); print('v$v s$s', d['tile'], d['world'], max(d['wall_ms']) if isinstance(d['wall_ms'],list) else d['wall_ms'], d.get('eff_wall'))"
done; done
