set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03/icache; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/list.txt 2>&1 || true
grep -i "icache\|ifetch\|SQC_\|INST_ANY" $O/list.txt | head -60 > $O/list_ic.txt || true
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d $O/ic -o p --output-format csv -- python3 bench.py --config 2 --no-cpu-baseline --steps 2 --warmup 1 > /dev/null 2> $O/ic.err || echo icfail
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -d $O/sq -o p --output-format csv -- python3 bench.py --config 2 --no-cpu-baseline --steps 2 --warmup 1 > /dev/null 2> $O/sq.err || echo sqfail
echo ok
