#!/bin/bash
# A/B of a host-side environment knob on one config: rounds of bench.py with VAR=A and VAR=B
# interleaved, then one run with VAR=B and the CPU comparison.
#   bash tools/r02_ab_env.sh <outdir> <config> <VAR> <A> <B> [rounds]
set -e
cd $GRAFT_REPO_ROOT
O=$1; C=$2; V=$3; A=$4; B=$5; R=${6:-3}
mkdir -p $O
for r in $(seq $R); do
  for x in $A $B; do
    env $V=$x timeout -k 10 200 python3 bench.py --config $C --no-cpu-baseline > $O/c${C}_${V}_${x}_r$r.json 2> $O/err.log
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['roofline']['kernel_avg_ms'])" $O/c${C}_${V}_${x}_r$r.json
  done
done
env $V=$B timeout -k 10 300 python3 bench.py --config $C --cpu-seconds 5 --numpy-seconds 0 > $O/c${C}_${V}_${B}_cpu.json 2>> $O/err.log
tail -c 300 $O/c${C}_${V}_${B}_cpu.json
