# C4 A/B: child refs loaded only by lanes with a hit child (PRT_LAZY_REFS) vs eager 4th load.
#   bash tools/r04_lazy.sh <outdir>
set -e
O=${1:-gpurun_out/lazy}
mkdir -p $O
timeout -k 10 500 python tools/ab_builds.py --libs abtmp/libprt_base.so abtmp/libprt_lazy.so --config 4 --rounds 5 --launches 3 > $O/ab_c4.jsonl 2> $O/ab_c4.err
cat $O/ab_c4.jsonl
echo ok
