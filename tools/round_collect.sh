#!/bin/bash
# After tools/round_full.sh <dir> ran on the GPU box: merge its PMC passes into profiles/pmc.json
# and copy the rocprof summaries, counter CSVs, bench lines and test log into profiles/<dest>.
#   bash tools/round_collect.sh gpurun_out/round profiles/r04/final
set -e
SRC=$1; DST=$2
[ -d $SRC/prof_c2 ] && python tools/pmc_summary.py --dir $SRC/prof_c2 --key cornell_512x512x64spp_d8 > /dev/null
[ -d $SRC/prof_c4 ] && python tools/pmc_summary.py --dir $SRC/prof_c4 --key cubes_512x512x64spp_d8 > /dev/null
# configs 1 / 3 / 5 when the profile stage covered them
[ -d $SRC/prof_c1 ] && python tools/pmc_summary.py --dir $SRC/prof_c1 --key cornell_128x128x4spp_d4 > /dev/null
[ -d $SRC/prof_c3 ] && python tools/pmc_summary.py --dir $SRC/prof_c3 --key specular_1024x1024x256spp_d8 > /dev/null
[ -d $SRC/prof_c5 ] && python tools/pmc_summary.py --dir $SRC/prof_c5 --key cornell_4096x4096x256spp_d8 > /dev/null
for c in prof_c1 prof_c2 prof_c3 prof_c4 prof_c5; do
  [ -d $SRC/$c ] || continue
  rm -rf $DST/$c; mkdir -p $DST/$c/fetch $DST/$c/write $DST/$c/sq
  cp $SRC/$c/bench.json $SRC/$c/bench_under_rocprof.json $DST/$c/
  cp $SRC/$c/trace/k_kernel_stats.csv $DST/$c/kernel_stats.csv
  for p in fetch write sq; do cp $SRC/$c/$p/*counter_collection.csv $DST/$c/$p/; done
done
if [ -d $SRC/bench_all ]; then mkdir -p $DST/bench_all && cp $SRC/bench_all/c*.json $DST/bench_all/; fi
[ -f $SRC/pytest_gpu.log ] && cp $SRC/pytest_gpu.log $DST/
python - "$SRC" <<'PY'
import json, os, sys
src = sys.argv[1]
for c in range(1, 6):
    import os
    if not os.path.exists(f'{src}/bench_all/c{c}.json'):
        continue
    d = json.loads(open(f'{src}/bench_all/c{c}.json').read().strip().splitlines()[-1]); r = d['roofline']
    print(c, d['value'], d['ms_per_step'], r['bound'], r.get('frac'), r.get('kernel_avg_ms'), (d['cpu_baseline'] or {}).get('value'))
d = json.load(open('profiles/pmc.json'))
for k, v in d.items():
    print(k, v['kernel_sha'], v['valu_issue_util'], v['valu_lane_util'], round(v['hbm_bytes_per_launch'] / 1e9, 3),
          round(v['hbm_bytes_raw'] / 1e9, 3), v['dispatch_ms'])
for c in (2, 4):
    if not os.path.exists(f'{src}/prof_c{c}/bench.json'):
        continue
    d = json.loads(open(f'{src}/prof_c{c}/bench.json').read().strip().splitlines()[-1])
    print('prof', c, d['value'], d['roofline']['kernel_avg_ms'])
    print(open(f'{src}/prof_c{c}/trace/k_kernel_stats.csv').read().splitlines()[1][:130])
PY
