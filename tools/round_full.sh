# Full check of the current build on one GPU: every -m gpu test, rocprofv3 + PMC passes for
# configs 2 and 4 (tools/profile_bench.sh), one bench line per BASELINE config.
#   bash tools/round_full.sh <outdir>
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/round}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -3 $O/pytest_gpu.log
bash tools/profile_bench.sh 2 $O/prof_c2
bash tools/profile_bench.sh 4 $O/prof_c4
bash tools/bench_all.sh $O/bench_all
echo ok
