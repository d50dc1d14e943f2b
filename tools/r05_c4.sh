#!/bin/bash
# Round 5: config 4 with the SBVH build (default) against the object-split build (PRT_SBVH=0), interleaved,
# plus the C4 GPU tests on the SBVH tree.
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/c4}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 500 --timeout-method thread -k "config4" > $O/pytest_c4.log 2>&1
tail -2 $O/pytest_c4.log
for r in 1 2; do
for kv in PRT_SBVH=1 PRT_SBVH=0; do
  env $kv timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline --numpy-seconds 0 --single-frame-steps 0 > "$O/c4_${kv}_r$r.json" 2> $O/c4.err
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['roofline']['kernel_avg_ms'], d['work_per_sample'], d['config']['scene_build_s'])" "$O/c4_${kv}_r$r.json"
done
done
echo ok
