# shard_sim at this build: frames per launch 1 (3 in flight) vs 8 / 16 (serial launches), gather proxy on
# torch's collective-stream ordering.  bash tools/r04_shard.sh <outdir>
set -e
O=${1:-gpurun_out/shard}
mkdir -p $O
S="timeout -k 10 300 python tools/shard_sim.py --config 2 --tiles 16 --schemes latin --worlds 2,4,8 --proxy stream"
$S --streams 3 --frames 1 --steps 12 > $O/f1_s3.jsonl 2> $O/f1_s3.err; cat $O/f1_s3.jsonl
$S --streams 1 --frames 8 --steps 16 > $O/f8.jsonl 2> $O/f8.err; cat $O/f8.jsonl
$S --streams 1 --frames 16 --steps 32 > $O/f16.jsonl 2> $O/f16.err; cat $O/f16.jsonl
$S --streams 2 --frames 8 --steps 16 > $O/f8_s2.jsonl 2> $O/f8_s2.err; cat $O/f8_s2.jsonl
