set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/s3ab1
mkdir -p $O
L="abtmp/libprt_base.so abtmp/libprt_nan.so abtmp/libprt_sqrt.so abtmp/libprt_push.so abtmp/libprt_all.so"
timeout -k 10 200 python tools/ab_builds.py --libs $L --config 2 --rounds 6 > $O/c2.log 2>&1
timeout -k 10 300 python tools/ab_builds.py --libs $L --config 4 --rounds 4 --launches 3 > $O/c4.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VSKIPPED SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 -d $O/mixa -o p --output-format csv -- python3 tools/one_render.py --config 2 > $O/mixa.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU_CVT SQ_INST_CYCLES_SALU SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_INSTS_VALU_INT64 -d $O/mixb -o p --output-format csv -- python3 tools/one_render.py --config 2 > $O/mixb.log 2>&1
echo ok
