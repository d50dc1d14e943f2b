set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/s3ab6
mkdir -p $O
L="abtmp/libprt_oct.so abtmp/libprt_oct2.so abtmp/libprt_oct3.so"
timeout -k 10 200 python tools/ab_builds.py --libs $L --config 2 --rounds 6 > $O/c2.log 2>&1
timeout -k 10 300 python tools/ab_builds.py --libs $L --config 4 --rounds 3 --launches 3 > $O/c4.log 2>&1
echo ok
