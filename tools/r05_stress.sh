#!/bin/bash
# Round 5: repeated full-frame renders of the pooled kernel's schedules with block-level
# synchronisation (fused 9, packed 11, split arrival 13 / 14) against the default 7; every frame
# must be bit-identical to the first (tools/ab_variants.py), configs 2 and 3.
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/stress}
mkdir -p $O
timeout -k 10 400 python -u tools/ab_variants.py --rounds 8 --variants 7 9 11 13 14 > $O/c2.jsonl 2> $O/c2.err
grep -c '"identical_to_first": true' $O/c2.jsonl
timeout -k 10 400 python -u tools/ab_variants.py --scene specular --res 1024 --spp 32 --rounds 3 --variants 7 9 11 13 14 > $O/c3.jsonl 2> $O/c3.err
grep -c '"identical_to_first": true' $O/c3.jsonl
echo ok
