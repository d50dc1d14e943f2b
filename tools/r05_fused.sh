#!/bin/bash
# Round 5: the fused pooled schedule (variants 9 / 10) against the two-phase pooled kernel (7 / 8):
# GPU parity tests, interleaved variant A/B at configs 2 and 3, lane table, bench lines.
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/fused}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frames.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/ab_variants.py --rounds 5 --variants 7 9 10 8 > $O/ab_c2.jsonl 2> $O/ab_c2.err
cat $O/ab_c2.jsonl
timeout -k 10 300 python -u tools/ab_variants.py --scene specular --res 1024 --spp 32 --rounds 3 --variants 7 9 10 > $O/ab_c3.jsonl 2> $O/ab_c3.err
tail -3 $O/ab_c3.jsonl
timeout -k 10 120 python -u tools/lane_table.py --config 2 --variant 9 > $O/lanes_c2_v9.json 2> $O/lanes.err
cat $O/lanes_c2_v9.json
timeout -k 10 200 python -u bench.py --no-cpu-baseline --variant 9 > $O/bench_v9.json 2> $O/bench_v9.err
timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/bench_v7.json 2> $O/bench_v7.err
python -c "import json;[print(f, json.load(open('$O/'+f))['value']) for f in ('bench_v9.json','bench_v7.json')]"
echo ok
