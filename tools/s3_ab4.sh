set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/s3ab4
mkdir -p $O
timeout -k 10 200 python tools/ab_builds.py --libs abtmp/libprt_new3.so abtmp/libprt_rayhack.so --config 2 --rounds 6 > $O/c2.log 2>&1
echo ok
