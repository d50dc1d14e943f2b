set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/s3ab3
mkdir -p $O
timeout -k 10 200 python tools/ab_variants.py --res 512 --spp 64 --depth 8 --rounds 5 --variants 1 6 > $O/c2_w7.log 2>&1
echo ok
