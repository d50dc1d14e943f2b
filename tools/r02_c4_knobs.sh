set -e
cd $GRAFT_REPO_ROOT
run() { echo "$1" >> gpurun_out/r02_c4_knobs.log; env $1 timeout -k 10 200 python tools/ab_variants.py --scene cubes --res 512 --spp 64 --depth 8 --rounds 2 --variants 3 2>&1 | grep kernel_ms >> gpurun_out/r02_c4_knobs.log; }
run "PRT_X=0"
run "PRT_RESUME_MIN=32"
run "PRT_RESUME_MIN=56"
run "PRT_LEAF_BREAK=4"
run "PRT_LEAF_BREAK=16"
run "PRT_LEAF_EXIT=4"
run "PRT_LEAF_EXIT=16"
run "PRT_X=1"
