set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/s3ab9
mkdir -p $O
timeout -k 10 300 python tools/ab_builds.py --libs abtmp/libprt_d2.so abtmp/libprt_pf.so --config 4 --rounds 5 --launches 3 > $O/c4.log 2>&1
echo ok
