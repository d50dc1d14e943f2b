# Pooled kernel without the in-kernel camera path (half the SGPR spills) vs with it, C2 and C3 (1024^2 x 32 spp
# via ab_builds' config 3 at full size is long; config 2 plus a second round).  bash tools/r04_nocam.sh <outdir>
set -e
O=${1:-gpurun_out/nocam}
mkdir -p $O
timeout -k 10 300 python tools/ab_builds.py --libs abtmp/libprt_base.so abtmp/libprt_nocam.so --config 2 --rounds 6 --launches 6 > $O/ab_c2.jsonl 2> $O/ab_c2.err
cat $O/ab_c2.jsonl
timeout -k 10 300 python tools/ab_builds.py --libs abtmp/libprt_nocam.so abtmp/libprt_base.so --config 2 --rounds 6 --launches 6 > $O/ab_c2_rev.jsonl 2> $O/ab_c2_rev.err
cat $O/ab_c2_rev.jsonl
echo ok
