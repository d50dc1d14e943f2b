set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/s3ab8
mkdir -p $O
timeout -k 10 200 python tools/ab_builds.py --libs abtmp/libprt_d1.so abtmp/libprt_nonz.so --config 2 --rounds 8 > $O/c2_nonz.log 2>&1
for le in 4 8 12 16; do echo "leaf_exit $le" >> $O/c2_le.log; PRT_LEAF_EXIT=$le timeout -k 10 200 python tools/ab_variants.py --res 512 --spp 64 --depth 8 --rounds 4 --variants 1 >> $O/c2_le.log 2>&1; done
for ml in 2 3 4 6 8; do echo "max_leaf $ml" >> $O/c2_ml.log; PRT_MAX_LEAF=$ml timeout -k 10 200 python tools/ab_variants.py --res 512 --spp 64 --depth 8 --rounds 4 --variants 1 >> $O/c2_ml.log 2>&1; done
echo ok
