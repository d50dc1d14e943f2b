#!/bin/bash
# A/B of libraries under abtmp/ on configs 2 and 4 (tools/ab_builds.py), one GPU.
#   bash tools/r02_ab.sh <outdir> <lib1> <lib2> [...]
set -e
cd $GRAFT_REPO_ROOT
O=$1; shift
mkdir -p $O
timeout -k 10 240 python tools/ab_builds.py --libs "$@" --config 2 --rounds 5 > $O/c2.log 2>&1
timeout -k 10 300 python tools/ab_builds.py --libs "$@" --config 4 --rounds 4 --launches 3 > $O/c4.log 2>&1
cat $O/c2.log $O/c4.log | grep lib
