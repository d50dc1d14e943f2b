# C4 node format A/B (64-B quantised vs compact 48-B records, + triangle-load pipelining) and the
# global-scene GPU tests at the compact format.   bash tools/r04_c4ab.sh <outdir>
set -e
O=${1:-gpurun_out/c4ab}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_hits.py -x -v --timeout 300 --timeout-method thread > $O/pytest_c4.log 2>&1
tail -3 $O/pytest_c4.log
timeout -k 10 400 python tools/ab_builds.py --libs abtmp/libprt_qn64.so abtmp/libprt_c48.so abtmp/libprt_c48_tp.so --config 4 --rounds 4 --launches 3 > $O/ab_c4.jsonl 2> $O/ab_c4.err
cat $O/ab_c4.jsonl
timeout -k 10 200 python bench.py --config 4 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err
tail -c 400 $O/bench_c4.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "variants or full_size or mis" > $O/pytest_var9.log 2>&1
tail -2 $O/pytest_var9.log
timeout -k 10 300 python tools/ab_variants.py --res 512 --spp 64 --depth 8 --rounds 5 --variants 7 9 > $O/ab_var79_c2.jsonl 2> $O/ab_var79_c2.err
cat $O/ab_var79_c2.jsonl
timeout -k 10 300 python tools/ab_variants.py --scene specular --res 1024 --spp 32 --depth 8 --rounds 3 --variants 7 9 > $O/ab_var79_c3.jsonl 2> $O/ab_var79_c3.err
cat $O/ab_var79_c3.jsonl
