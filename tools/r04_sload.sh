# Global-scene kernel: a node visit whose active lanes all sit on one node loads it with one scalar
# 64-B load (constant cache) instead of four vector loads through the L1, vs the base (C4, both
# orders; images must be identical).   bash tools/r04_sload.sh <outdir>
set -e
O=${1:-gpurun_out/sload}
mkdir -p $O
timeout -k 10 300 python tools/ab_builds.py --libs abtmp/libprt_base.so abtmp/libprt_sload.so --config 4 --rounds 4 --launches 3 > $O/ab_c4.jsonl 2> $O/ab_c4.err
cat $O/ab_c4.jsonl
timeout -k 10 300 python tools/ab_builds.py --libs abtmp/libprt_sload.so abtmp/libprt_base.so --config 4 --rounds 4 --launches 3 > $O/ab_c4_rev.jsonl 2> $O/ab_c4_rev.err
cat $O/ab_c4_rev.jsonl
echo ok
