#!/bin/bash
# One-at-a-time sweep of the traversal knobs (env PRT_*) on one config, interleaved with the
# defaults:   bash tools/knob_sweep.sh <outdir> <config> [rounds] "VAR=value VAR=value,VAR2=value ..."
set -e
cd $GRAFT_REPO_ROOT
O=$1; C=$2; R=${3:-2}; SETS=${4:-"PRT_RESUME_MIN=16 PRT_RESUME_MIN=48 PRT_LEAF_BREAK=8 PRT_LEAF_BREAK=24 PRT_LEAF_EXIT=8 PRT_LEAF_EXIT=16"}
mkdir -p $O
for r in $(seq $R); do
  for kv in DEFAULT $SETS; do
    E=""; [ $kv != DEFAULT ] && E=${kv//,/ }
    env $E timeout -k 10 200 python3 bench.py --config $C --no-cpu-baseline --numpy-seconds 0 > $O/c${C}_${kv}_r$r.json 2> $O/err.log
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$kv r$r', d['value'], d['roofline']['kernel_avg_ms'], d.get('work_per_sample'))" $O/c${C}_${kv}_r$r.json
  done
done
