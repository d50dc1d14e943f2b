# Round 6 A/B of the working tree's libprt against abtmp/libprt_head.so (the last commit's build) in
# one process per config (tools/ab_builds.py: interleaved rounds, images must be identical), after the
# guard selftest and the GPU suite.
#   bash tools/r06_ab.sh <outdir> [configs...]
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/r06ab}; shift || true
CONFIGS=${@:-2 3 1}
mkdir -p $O
timeout -k 10 120 python -u -m pytest tests/test_gpu_selftest.py -x -q -s --timeout 100 --timeout-method thread > $O/selftest.log 2>&1
grep "guards" $O/selftest.log | head -2
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -2 $O/pytest_gpu.log
for c in $CONFIGS; do
  r=5; l=5; [ "$c" = 3 ] && { r=3; l=2; }
  timeout -k 10 300 python -u tools/ab_builds.py --libs abtmp/libprt_head.so pyrenderer_amd/lib/libprt.so --config $c --rounds $r --launches $l > $O/ab_c$c.jsonl 2> $O/ab_c$c.err
  cat $O/ab_c$c.jsonl
done
