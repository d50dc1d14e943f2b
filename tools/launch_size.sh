#!/bin/bash
# Throughput against launch size on one GPU (config 2's frame at fewer samples per pixel)
#   bash tools/launch_size.sh <outdir>
set -e
cd $GRAFT_REPO_ROOT
O=$1; mkdir -p $O
run() { n=$1; shift; timeout -k 10 200 python3 bench.py --config 2 --no-cpu-baseline --numpy-seconds 0 --steps 30 --warmup 5 "$@" > $O/$n.json 2> $O/$n.err;
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline'].get('variant', ''))"; }
run full_s1_t64 --spp 64 --streams 1 --tile 64
run full_s3_t16 --spp 64 --streams 3 --tile 16
run spp8_s3_t16 --spp 8 --streams 3 --tile 16
run spp8_s3_t16_v7 --spp 8 --streams 3 --tile 16 --variant 7
run spp8_s1_t64 --spp 8 --streams 1 --tile 64
run spp8_s3_t64 --spp 8 --streams 3 --tile 64
run spp16_s3_t16 --spp 16 --streams 3 --tile 16
run spp32_s2_t16 --spp 32 --streams 2 --tile 16
