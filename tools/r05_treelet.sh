#!/bin/bash
# Round 5: treelet restructuring of the BVH2 (PRT_TREELET passes) at config 4, interleaved with the
# default build at configs 4 and 2, plus the C4 parity tests on the restructured tree.
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/treelet}
mkdir -p $O
PRT_TREELET=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "config4" > $O/pytest_c4.log 2>&1 || { tail -20 $O/pytest_c4.log; exit 1; }
tail -2 $O/pytest_c4.log
bash tools/knob_sweep.sh $O 4 2 "PRT_TREELET=1 PRT_TREELET=3 PRT_TREELET=3,PRT_SAH_CT=0.3"
bash tools/knob_sweep.sh $O 2 3 "PRT_TREELET=3"
echo ok
