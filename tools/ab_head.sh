set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/headab
timeout -k 10 300 python -u tools/ab_builds.py --libs abtmp/libprt_head.so pyrenderer_amd/lib/libprt.so --config 2 --rounds 5 --launches 5 > gpurun_out/headab/c2.jsonl 2> gpurun_out/headab/c2.err
timeout -k 10 300 python -u tools/ab_builds.py --libs pyrenderer_amd/lib/libprt.so abtmp/libprt_head.so --config 3 --rounds 3 --launches 2 > gpurun_out/headab/c3.jsonl 2> gpurun_out/headab/c3.err
cat gpurun_out/headab/c2.jsonl gpurun_out/headab/c3.jsonl
