set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "variants or soup" --timeout 200 --timeout-method thread > gpurun_out/r02_bvh8_tests.log 2>&1
timeout -k 10 300 python tools/ab_variants.py --scene cubes --res 512 --spp 64 --depth 8 --rounds 3 --variants 3 8 > gpurun_out/r02_ab8_c4.log 2>&1
timeout -k 10 300 python tools/ab_variants.py --scene soup:200000 --res 512 --spp 16 --depth 8 --rounds 3 --variants 3 8 > gpurun_out/r02_ab8_soup.log 2>&1
