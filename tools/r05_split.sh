#!/bin/bash
# Round 5: the pooled kernel without the block barrier (split arrival, variants 13 / 14) against the
# two-phase pooled kernel (7 / 8): GPU parity of every variant, interleaved variant A/B at configs 2 and 3.
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/split}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frames.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/ab_variants.py --rounds 5 --variants 7 13 14 8 > $O/ab_c2.jsonl 2> $O/ab_c2.err
cat $O/ab_c2.jsonl
timeout -k 10 300 python -u tools/ab_variants.py --scene specular --res 1024 --spp 32 --rounds 3 --variants 7 13 > $O/ab_c3.jsonl 2> $O/ab_c3.err
tail -2 $O/ab_c3.jsonl
echo ok
