set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03/npk; mkdir -p $O
for r in 1 2; do for f in "" "--no-primary-kernel"; do
  timeout -k 10 200 python3 bench.py --config 2 --no-cpu-baseline --numpy-seconds 0 $f > $O/c2_${r}_${f:2:2}.json 2> $O/err.log
  python3 -c "import json; d=json.loads(open('$O/c2_${r}_${f:2:2}.json').read().strip().splitlines()[-1]); print('c2 $f', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])"
  timeout -k 10 200 python3 bench.py --config 3 --no-cpu-baseline --numpy-seconds 0 --steps 3 --warmup 1 $f > $O/c3_${r}_${f:2:2}.json 2> $O/err.log
  python3 -c "import json; d=json.loads(open('$O/c3_${r}_${f:2:2}.json').read().strip().splitlines()[-1]); print('c3 $f', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])"
done; done
