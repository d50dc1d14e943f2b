set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/s4
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -3 $O/pytest_gpu.log
bash tools/profile_bench.sh 2 $O/prof_c2
echo ok
