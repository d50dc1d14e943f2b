# Round-end evidence for the current build, in two gpurun calls (each well inside the 20-minute cap):
#   bash tools/r04_final.sh <outdir> a   every -m gpu test, rocprofv3 + PMC passes for configs 2 and 4,
#                                        one bench line per config
#   bash tools/r04_final.sh <outdir> b   rocprofv3 + PMC passes for configs 1, 3, 5 and the
#                                        memory-pipeline counters of C2 / C4
# then, here: bash tools/round_collect.sh <outdir> profiles/r04/final
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/final}
mkdir -p $O
if [ "${2:-a}" = a ]; then
  timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  tail -3 $O/pytest_gpu.log
  for c in 2 4; do bash tools/profile_bench.sh $c $O/prof_c$c; done
  bash tools/bench_all.sh $O/bench_all
else
  timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_frames.log 2>&1
  tail -2 $O/pytest_frames.log
  for c in 1 3 5; do bash tools/profile_bench.sh $c $O/prof_c$c; done
  bash tools/pmc_mem.sh 2 $O/pmc_mem_c2
  bash tools/pmc_mem.sh 4 $O/pmc_mem_c4
  timeout -k 10 300 python tools/shard_sim.py --config 2 --tiles 16 --schemes latin --worlds 2,4,8 --proxy stream \
    --streams 1 --frames 16 --steps 32 > $O/shard_f16.jsonl 2> $O/shard_f16.err
  cat $O/shard_f16.jsonl
fi
echo ok
