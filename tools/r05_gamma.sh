#!/bin/bash
# Round 5: the LDS kernels' slab test without the 1 + 2 gamma_3 factor on t_far (the box padding
# alone keeps it conservative), against the default build: images identical, configs 2 and 3.
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/gamma}
mkdir -p $O
timeout -k 10 300 python -u tools/ab_builds.py --libs pyrenderer_amd/lib/libprt.so abtmp/libprt_nogamma.so --config 2 --rounds 5 --launches 5 > $O/ab_c2.jsonl 2> $O/ab_c2.err
cat $O/ab_c2.jsonl
timeout -k 10 300 python -u tools/ab_builds.py --libs abtmp/libprt_nogamma.so pyrenderer_amd/lib/libprt.so --config 2 --rounds 5 --launches 5 > $O/ab_c2_rev.jsonl 2> $O/ab_c2_rev.err
cat $O/ab_c2_rev.jsonl
timeout -k 10 300 python -u tools/ab_builds.py --libs pyrenderer_amd/lib/libprt.so abtmp/libprt_nogamma.so --config 3 --rounds 3 --launches 1 > $O/ab_c3.jsonl 2> $O/ab_c3.err
cat $O/ab_c3.jsonl
echo ok
