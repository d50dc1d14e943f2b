set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/s3ab7
mkdir -p $O
timeout -k 10 300 python tools/ab_builds.py --libs abtmp/libprt_oct3.so abtmp/libprt_oct2.so abtmp/libprt_oct.so --config 2 --rounds 10 > $O/c2.log 2>&1
timeout -k 10 300 python tools/ab_builds.py --libs abtmp/libprt_oct3.so abtmp/libprt_oct.so --config 3 --rounds 3 --launches 2 > $O/c3.log 2>&1
echo ok
