# Concurrency probe: one process, multi-frame launches on 1 / 2 / 3 streams (does a second
# persistent launch in flight add throughput?), and 2 / 4 gloo ranks sharing the GPU.
#   bash tools/r04_conc.sh <outdir>
set -e
O=${1:-gpurun_out/conc}
mkdir -p $O
for r in 1 2; do
for s in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 24 --warmup 8 --frames-per-launch 8 --streams $s --no-cpu-baseline > $O/s${s}_r$r.json 2> $O/s${s}_r$r.err
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('streams $s r$r', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])" $O/s${s}_r$r.json
done
done
timeout -k 10 200 python bench.py --steps 24 --warmup 8 --frames-per-launch 8 --tile 16 --no-cpu-baseline > $O/t16.json 2> $O/t16.err
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('tile16', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])" $O/t16.json
for n in 4 2; do
  timeout -k 10 300 python bench.py --gpus $n --backend gloo --steps 24 --warmup 8 --frames-per-launch 8 --no-cpu-baseline > $O/gloo_n$n.json 2> $O/gloo_n$n.err
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('gloo $n', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])" $O/gloo_n$n.json
done
echo ok
