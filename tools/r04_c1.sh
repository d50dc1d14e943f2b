# Config 1 at this build's auto frames per launch (256 frames of 65 k samples): bench line + profile.
#   bash tools/r04_c1.sh <outdir>
set -e
O=${1:-gpurun_out/c1}
mkdir -p $O/bench_all
timeout -k 10 400 python3 bench.py --config 1 --steps 400 --warmup 20 > $O/bench_all/c1.json 2> $O/bench_all/c1.err
tail -c 300 $O/bench_all/c1.json
bash tools/profile_bench.sh 1 $O/prof_c1
echo ok
