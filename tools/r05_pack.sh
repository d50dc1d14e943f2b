#!/bin/bash
# Round 5: packed leaf trips (variants 11 / 12, traverse_pk) against the two-phase pooled kernel (7 / 8):
# GPU parity of every variant, interleaved variant A/B at configs 2 and 3, lane table.
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/pack}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "variants or config2 or pool" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/ab_variants.py --rounds 5 --variants 7 11 12 8 > $O/ab_c2.jsonl 2> $O/ab_c2.err
cat $O/ab_c2.jsonl
timeout -k 10 120 python -u tools/lane_table.py --config 2 --variant 11 > $O/lanes_c2_v11.json 2> $O/lanes.err
cat $O/lanes_c2_v11.json
timeout -k 10 300 python -u tools/ab_variants.py --scene specular --res 1024 --spp 32 --rounds 3 --variants 7 11 > $O/ab_c3.jsonl 2> $O/ab_c3.err
tail -3 $O/ab_c3.jsonl
if [ -f abtmp/libprt_h3.so ]; then
  timeout -k 10 300 python -u tools/ab_builds.py --libs pyrenderer_amd/lib/libprt.so abtmp/libprt_h1.so abtmp/libprt_h3.so --config 2 --rounds 4 --launches 4 --variant 11 > $O/ab_hold.jsonl 2> $O/ab_hold.err
  tail -4 $O/ab_hold.jsonl
fi
echo ok
