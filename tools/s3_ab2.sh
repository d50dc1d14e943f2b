set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/s3ab2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hits.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python tools/ab_builds.py --libs abtmp/libprt_base.so abtmp/libprt_new2.so --config 2 --rounds 6 > $O/c2.log 2>&1
for k in 32 85 128 160; do echo "lds_top $k" >> $O/c4_top.log; PRT_LDS_TOP=$k timeout -k 10 300 python tools/ab_variants.py --scene cubes --res 512 --spp 64 --depth 8 --rounds 3 --variants 3 6 >> $O/c4_top.log 2>&1; done
echo ok
