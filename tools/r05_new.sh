#!/bin/bash
# Round 5: GPU tests of this round's host/ABI additions + the full GPU suite + a default bench line.
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/new}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_camera.py tests/test_gpu_frames.py tests/test_gpu_boundary.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_new.log 2>&1
tail -3 $O/pytest_new.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['single_frame'], d['config']['ranks'], d['rank_ms_per_step'])"
echo ok1
# config 4: object-split BVH vs spatial splits (SBVH, env PRT_SBVH=1): work counters + kernel time
for kv in PRT_SBVH=0 "PRT_SBVH=1 PRT_SBVH_ALPHA=1e-3"; do
  env $kv timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline --numpy-seconds 0 --single-frame-steps 0 > "$O/c4_${kv// /_}.json" 2> $O/c4.err
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['roofline']['kernel_avg_ms'], d['work_per_sample'], d['config']['scene_build_s'])" "$O/c4_${kv// /_}.json"
done
echo ok2
