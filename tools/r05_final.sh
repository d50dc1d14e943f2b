#!/bin/bash
# Round-end evidence for the current build, in two gpurun calls:
#   bash tools/r05_final.sh <outdir> a   every -m gpu test; rocprofv3 kernel trace + PMC passes for configs 1-5
#   (here: bash tools/round_collect.sh <outdir> profiles/r05/final — merges the PMC into profiles/pmc.json)
#   bash tools/r05_final.sh <outdir> b   one bench line per config (reading this build's PMC entries), the
#                                        memory-pipeline counters of C2 / C4, the 8-rank shard simulation
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/final}
mkdir -p $O
if [ "${2:-a}" = a ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1
  tail -3 $O/pytest_gpu.log
  for c in 2 4 1 3 5; do bash tools/profile_bench.sh $c $O/prof_c$c; done
else
  bash tools/bench_all.sh $O/bench_all
  bash tools/pmc_mem.sh 2 $O/pmc_mem_c2
  bash tools/pmc_mem.sh 4 $O/pmc_mem_c4
  timeout -k 10 300 python tools/shard_sim.py --config 2 --tiles 16 --schemes latin --worlds 2,4,8 --proxy stream \
    --streams 1 --frames 16 --steps 32 > $O/shard_f16.jsonl 2> $O/shard_f16.err
  cat $O/shard_f16.jsonl
fi
echo ok
