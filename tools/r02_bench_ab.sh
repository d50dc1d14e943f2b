#!/bin/bash
# A/B whole bench steps (camera + trace + reduce kernels) of library copies: each round copies a
# library over pyrenderer_amd/lib/libprt.so (in the GPU box's scratch copy of the tree) and runs
# bench.py --config C without the CPU legs.   bash tools/r02_bench_ab.sh <outdir> <config> <libs...>
set -e
cd $GRAFT_REPO_ROOT
O=$1; C=$2; shift 2
mkdir -p $O
cp pyrenderer_amd/lib/libprt.so $O/.orig.so
for r in 1 2 3; do
  for L in "$@"; do
    cp $L pyrenderer_amd/lib/libprt.so
    timeout -k 10 120 python bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'lib': '$L', 'round': $r, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['roofline']['kernel_avg_ms']}))" >> $O/bench_ab.jsonl
  done
done
cp $O/.orig.so pyrenderer_amd/lib/libprt.so
cat $O/bench_ab.jsonl
