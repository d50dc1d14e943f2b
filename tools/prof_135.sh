#!/bin/bash
# rocprofv3 kernel-trace summary + PMC passes for configs 1, 3 and 5 (tools/profile_bench.sh),
# so that every BASELINE config's bench line carries measured traffic and VALU figures.
#   bash tools/prof_135.sh <outdir>
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/prof135}
for c in 1 3 5; do bash tools/profile_bench.sh $c $O/prof_c$c; done
for c in 1 3 5; do timeout -k 10 400 python3 bench.py --config $c $( [ $c = 1 ] && echo --steps 400 --warmup 20 ) --no-cpu-baseline > $O/recheck_c$c.json 2> $O/recheck_c$c.err || true; done
echo ok
