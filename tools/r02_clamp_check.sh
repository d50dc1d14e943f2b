set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_pytest_clamp.log 2>&1
timeout -k 10 300 python tools/ab_builds.py --libs abtmp/libprt_escnan.so abtmp/libprt_clamp.so --config 4 --rounds 4 > gpurun_out/r02_ab_clamp_c4.log 2>&1
timeout -k 10 200 python tools/ab_builds.py --libs abtmp/libprt_escnan.so abtmp/libprt_clamp.so --config 2 --rounds 5 > gpurun_out/r02_ab_clamp_c2.log 2>&1
timeout -k 10 200 python tools/outlier_queries.py > gpurun_out/r02_outliers_c4_clamp.log 2>&1
timeout -k 10 200 python tools/wave_clock.py --config 4 > gpurun_out/r02_wclk_c4_clamp.log 2>&1
