set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/s4
mkdir -p $O
bash tools/profile_bench.sh 4 $O/prof_c4
bash tools/bench_all.sh $O/bench_all
echo ok
