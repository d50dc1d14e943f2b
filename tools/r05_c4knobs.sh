#!/bin/bash
# Round 5: config 4 knobs on the spatial-split tree (leaf-phase thresholds, resume threshold, SAH
# leaf cost, leaf size), interleaved with the defaults (tools/knob_sweep.sh).
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/c4knobs}
bash tools/knob_sweep.sh $O 4 2 "PRT_LEAF_BREAK=8 PRT_LEAF_BREAK=24 PRT_LEAF_EXIT=16 PRT_LEAF_EXIT=32 PRT_RESUME_MIN=24 PRT_RESUME_MIN=48 PRT_SAH_CT=0.3 PRT_SAH_CT=1.0 PRT_MAX_LEAF=2 PRT_SBVH_BUDGET=2 PRT_SBVH_ALPHA=1e-6"
echo ok
