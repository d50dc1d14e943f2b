set -o pipefail
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -5 $O/pytest_gpu.log
[ $rc = 0 ] || exit $rc
timeout -k 10 200 python bench.py --frames-per-launch 1 --no-cpu-baseline > $O/bench_f1.json 2> $O/bench_f1.err && tail -c 300 $O/bench_f1.json &&
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err && tail -c 1500 $O/bench.json &&
timeout -k 10 200 python bench.py --frames-per-launch 1 --no-cpu-baseline > $O/bench_f1b.json 2> $O/bench_f1b.err && tail -c 300 $O/bench_f1b.json &&
timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline > $O/bench_s20.json 2> $O/bench_s20.err && tail -c 300 $O/bench_s20.json
