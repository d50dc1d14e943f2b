set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "variants or spill or mis or full_size" --timeout 200 --timeout-method thread > gpurun_out/r02_spread_tests.log 2>&1
timeout -k 10 200 python tools/ab_variants.py --res 512 --spp 64 --depth 8 --rounds 5 --variants 1 6 > gpurun_out/r02_ab_c2.log 2>&1
for le in 0 2 16 32; do echo "leaf_exit $le" >> gpurun_out/r02_ab_c2_le.log; PRT_LEAF_EXIT=$le timeout -k 10 200 python tools/ab_variants.py --res 512 --spp 64 --depth 8 --rounds 3 --variants 1 6 >> gpurun_out/r02_ab_c2_le.log 2>&1; done
timeout -k 10 300 python tools/ab_variants.py --scene cubes --res 512 --spp 64 --depth 8 --rounds 3 --variants 3 7 > gpurun_out/r02_ab_c4.log 2>&1
