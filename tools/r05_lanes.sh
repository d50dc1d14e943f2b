#!/bin/bash
# Round 5: per-phase lane table of the pooled kernel (tools/lane_table.py) for configs 2, 3, 1, with the
# wave-cycle split of a -D PRT_POOL_CLOCKS copy (abtmp/libprt_clk.so), plus a default bench line.
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/lanes}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_parity.log 2>&1
tail -2 $O/pytest_parity.log
timeout -k 10 120 python -u tools/lane_table.py --config 2 --clocks abtmp/libprt_clk.so > $O/c2.json 2> $O/c2.err
cat $O/c2.json
timeout -k 10 200 python -u tools/lane_table.py --config 3 --clocks abtmp/libprt_clk.so > $O/c3.json 2> $O/c3.err
timeout -k 10 120 python -u tools/lane_table.py --config 1 > $O/c1.json 2> $O/c1.err
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err
cat $O/bench_c2.json
echo ok
