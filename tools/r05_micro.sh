#!/bin/bash
# Round 5: 32-bit (v_mad_u32_u24) vs 64-bit flat (v_mad_u64_u32) addressing of the LDS scene copy in
# the pooled / LDS kernels, interleaved A/B at configs 2 and 3; VALU op-rate probe.
set -e
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/micro}
mkdir -p $O



timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/ab_builds.py --libs pyrenderer_amd/lib/libprt.so abtmp/libprt_noaddr32.so --rounds 6 > $O/ab_c2.jsonl 2> $O/ab.err
cut -c1-150 $O/ab_c2.jsonl
timeout -k 10 300 python -u tools/ab_builds.py --libs pyrenderer_amd/lib/libprt.so abtmp/libprt_noaddr32.so --rounds 3 --config 3 --launches 1 > $O/ab_c3.jsonl 2> $O/ab3.err
cut -c1-150 $O/ab_c3.jsonl
echo ok
