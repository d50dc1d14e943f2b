set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/s3ab5
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hits.py tests/test_multi_light.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python tools/ab_builds.py --libs abtmp/libprt_new3.so abtmp/libprt_oct.so --config 2 --rounds 6 > $O/c2.log 2>&1
timeout -k 10 200 python tools/ab_builds.py --libs abtmp/libprt_new3.so abtmp/libprt_oct.so --config 3 --rounds 3 --launches 2 > $O/c3.log 2>&1
echo ok
