set -e
cd $GRAFT_REPO_ROOT
run() { echo "$1" >> gpurun_out/r02_c4_resume.log; env $1 timeout -k 10 200 python tools/ab_variants.py --scene cubes --res 512 --spp 64 --depth 8 --rounds 3 --variants 3 2>&1 | grep kernel_ms >> gpurun_out/r02_c4_resume.log; }
run "PRT_RESUME_MIN=48"
run "PRT_RESUME_MIN=16"
run "PRT_RESUME_MIN=24"
run "PRT_RESUME_MIN=32"
run "PRT_RESUME_MIN=40"
run "PRT_RESUME_MIN=32 PRT_LEAF_BREAK=16"
run "PRT_RESUME_MIN=48"
