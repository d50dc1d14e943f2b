# Multi-GPU rehearsal on the one-GPU box at this build: shard_sim of C2 at 1 / 16 frames per launch
# (gather proxy on the collective-stream ordering), and bench.py --gpus N --backend gloo for N = 2, 4, 8
# (bench starts N ranks itself; all share the one GPU, so their value is NOT a scaling figure).
#   bash tools/r04_multi.sh <outdir>
set -e
O=${1:-gpurun_out/multi}
mkdir -p $O
S="timeout -k 10 300 python tools/shard_sim.py --config 2 --tiles 16 --schemes latin --worlds 2,4,8 --proxy stream"
$S --streams 3 --frames 1 --steps 12 > $O/shard_f1_s3.jsonl 2> $O/shard_f1_s3.err; cat $O/shard_f1_s3.jsonl
$S --streams 1 --frames 16 --steps 32 > $O/shard_f16.jsonl 2> $O/shard_f16.err; cat $O/shard_f16.jsonl
for n in 2 4 8; do
  timeout -k 10 300 python bench.py --gpus $n --backend gloo --steps 8 --warmup 1 --cpu-seconds 2 --numpy-seconds 0 > $O/bench_gloo_n$n.json 2> $O/bench_gloo_n$n.err
  tail -c 300 $O/bench_gloo_n$n.json
done
bash tools/profile_bench.sh 1 $O/prof_c1
echo ok
