#!/bin/bash
# Round 5: fused schedule with one visiting order (front to back for every lane) vs the per-lane order
# (abtmp/libprt_mixed.so) vs the two-phase kernel; leaf-phase knobs for the fused schedule.
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/fused2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "variants or pool or full_size" > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/ab_variants.py --rounds 5 --variants 7 9 > $O/ab_c2.jsonl 2> $O/ab_c2.err
tail -2 $O/ab_c2.jsonl
timeout -k 10 300 python -u tools/ab_builds.py --libs pyrenderer_amd/lib/libprt.so abtmp/libprt_mixed.so --variant 9 --rounds 4 > $O/ab_order.jsonl 2> $O/ab_order.err
cat $O/ab_order.jsonl | cut -c1-200
for kv in PRT_LEAF_EXIT=16 PRT_LEAF_EXIT=4 PRT_LEAF_BREAK=4 PRT_LEAF_BREAK=12; do
  env $kv timeout -k 10 300 python -u tools/ab_variants.py --rounds 3 --variants 7 9 > $O/knob_$kv.jsonl 2> $O/knob.err
  echo $kv; tail -2 $O/knob_$kv.jsonl | cut -c1-120
done
timeout -k 10 120 python -u tools/lane_table.py --config 2 --variant 9 > $O/lanes_c2_v9.json 2> $O/lanes.err
cat $O/lanes_c2_v9.json
echo ok
