# Lean pooled-kernel build for scenes without spheres / metal / dielectric (PLAIN) vs the one build
# for all scenes: C2 both orders, C3 (not plain: must be unchanged), the GPU tests touching the pool
# kernel; the global-scene kernel's lean build at 6 and 7 waves per SIMD against the base (C4).
#   bash tools/r04_plain.sh <outdir>
set -e
O=${1:-gpurun_out/plain}
mkdir -p $O
timeout -k 10 300 python tools/ab_builds.py --libs abtmp/libprt_base.so abtmp/libprt_plain.so --config 2 --rounds 6 --launches 6 > $O/ab_c2.jsonl 2> $O/ab_c2.err
cat $O/ab_c2.jsonl
timeout -k 10 300 python tools/ab_builds.py --libs abtmp/libprt_plain.so abtmp/libprt_base.so --config 2 --rounds 6 --launches 6 > $O/ab_c2_rev.jsonl 2> $O/ab_c2_rev.err
cat $O/ab_c2_rev.jsonl
timeout -k 10 300 python tools/ab_builds.py --libs abtmp/libprt_base.so abtmp/libprt_plain.so --config 3 --rounds 2 --launches 2 > $O/ab_c3.jsonl 2> $O/ab_c3.err
cat $O/ab_c3.jsonl
timeout -k 10 300 python tools/ab_builds.py --libs abtmp/libprt_base.so abtmp/libprt_gp6.so abtmp/libprt_gp7.so --config 4 --rounds 4 --launches 3 > $O/ab_c4.jsonl 2> $O/ab_c4.err
cat $O/ab_c4.jsonl
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_frames.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
echo ok
