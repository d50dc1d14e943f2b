# Leaf-phase knobs for the one-barrier pooled kernel at C2 (its thresholds were tuned on trace_kernel),
# and smoke().   bash tools/r04_knobs.sh <outdir>
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/knobs}
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; tail -2 $O/smoke.log
timeout -k 10 900 bash tools/knob_sweep.sh $O/c2 2 2 "PRT_LEAF_EXIT=0 PRT_LEAF_EXIT=4 PRT_LEAF_EXIT=16 PRT_LEAF_EXIT=64 PRT_LEAF_BREAK=4 PRT_LEAF_BREAK=16"
timeout -k 10 600 bash tools/r04_conc.sh $O/conc
echo ok
