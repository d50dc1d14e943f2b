set -e
cd $GRAFT_REPO_ROOT
for b in 8 16 32 128 512; do echo "beta $b" >> gpurun_out/r02_esc_sweep.log; PRT_ESC_BETA=$b timeout -k 10 300 python tools/ab_variants.py --scene cubes --res 512 --spp 64 --depth 8 --rounds 2 --variants 3 >> gpurun_out/r02_esc_sweep.log 2>&1; done
timeout -k 10 200 python tools/wave_clock.py --config 4 > gpurun_out/r02_wclk_c4_esc.log 2>&1
