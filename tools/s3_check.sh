set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s3/pytest.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/s3/bench_c2.json 2> gpurun_out/s3/bench_c2.err
echo ok
