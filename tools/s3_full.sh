set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/s3full
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
bash tools/profile_bench.sh 2 $O/prof_c2
bash tools/profile_bench.sh 4 $O/prof_c4
bash tools/bench_all.sh $O/bench_all
echo ok
