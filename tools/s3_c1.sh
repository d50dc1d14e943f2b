set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/s3c1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "lds_soup or variants" --timeout 200 --timeout-method thread > $O/test.log 2>&1
for s in 2 3 4 6; do timeout -k 10 200 python bench.py --config 1 --streams $s --no-cpu-baseline --steps 200 --warmup 20 > $O/c1_s$s.json 2>/dev/null; done
echo ok
