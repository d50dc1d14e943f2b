set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_pytest_full.log 2>&1
bash tools/profile_bench.sh 2 gpurun_out/r02_prof2_c2
bash tools/profile_bench.sh 4 gpurun_out/r02_prof2_c4
