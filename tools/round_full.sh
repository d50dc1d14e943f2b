#!/bin/bash
# The one GPU-session driver (round 6 folded the per-round session scripts tools/r04_*.sh /
# tools/r05_*.sh into it; their logs stay under profiles/r04/ and profiles/r05/).
#   bash tools/round_full.sh <outdir> <stage> [configs...]       (GPU box, repo root)
# stages:
#   tests     the guard selftest, then every -m gpu test
#   profile   bench line + rocprofv3 kernel trace + PMC passes per config (default 2 4 1 3 5; then, here:
#             bash tools/round_collect.sh <outdir> profiles/rNN/final merges the PMC into profiles/pmc.json)
#   bench     one bench line per BASELINE config (reading this build's PMC), the memory-pipeline counters
#             of C2 / C4 and the 8-rank shard simulation
#   ab        in-process A/B of this build against abtmp/libprt_head.so (the last commit's build, made with
#             `python -m pyrenderer_amd.build --out abtmp/libprt_head.so` in a worktree of HEAD) per config
#             (default 2 3 1), images must be identical
#   all       tests, then profile
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/round}; STAGE=${2:-all}
shift 2 || true
mkdir -p $O
case $STAGE in
  tests|all)
    timeout -k 10 120 python -u -m pytest tests/test_gpu_selftest.py -x -q -s --timeout 100 --timeout-method thread > $O/selftest.log 2>&1
    grep "guards" $O/selftest.log | head -1
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1
    tail -3 $O/pytest_gpu.log
    [ $STAGE = all ] || { echo ok; exit 0; } ;;
esac
case $STAGE in
  profile|all)
    for c in ${@:-2 4 1 3 5}; do bash tools/profile_bench.sh $c $O/prof_c$c; done ;;
  bench)
    bash tools/bench_all.sh $O/bench_all
    bash tools/pmc_mem.sh 2 $O/pmc_mem_c2
    bash tools/pmc_mem.sh 4 $O/pmc_mem_c4
    timeout -k 10 300 python tools/shard_sim.py --config 2 --tiles 16 --schemes latin --worlds 2,4,8 --proxy stream \
      --streams 1 --frames 16 --steps 32 > $O/shard_f16.jsonl 2> $O/shard_f16.err
    cat $O/shard_f16.jsonl ;;
  ab)
    for c in ${@:-2 3 1}; do
      r=5; l=5; [ "$c" = 3 ] && { r=3; l=2; }
      timeout -k 10 300 python -u tools/ab_builds.py --libs abtmp/libprt_head.so pyrenderer_amd/lib/libprt.so \
        --config $c --rounds $r --launches $l > $O/ab_c$c.jsonl 2> $O/ab_c$c.err
      cat $O/ab_c$c.jsonl
    done ;;
esac
echo ok
