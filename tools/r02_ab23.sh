#!/bin/bash
# A/B of library copies on configs 2 and 3 (LDS-resident scenes) + image check vs the oracle.
#   bash tools/r02_ab23.sh <outdir> <lib1> <lib2> [...]
set -e
cd $GRAFT_REPO_ROOT
O=$1; shift
mkdir -p $O
for L in "$@"; do timeout -k 10 120 python tools/lib_vs_oracle.py --lib $L >> $O/oracle.log 2>&1; done
timeout -k 10 240 python tools/ab_builds.py --libs "$@" --config 2 --rounds 5 > $O/c2.log 2>&1
timeout -k 10 300 python tools/ab_builds.py --libs "$@" --config 3 --rounds 3 --launches 2 > $O/c3.log 2>&1
grep lib $O/oracle.log $O/c2.log $O/c3.log
