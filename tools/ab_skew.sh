#!/bin/bash
# A/B: RX final-round skew (-DMODEM_RX_SKEW) against the base DEV_MIN build, C3 and C5 bench legs.
cd ${GRAFT_REPO_ROOT:-.}
echo "== c3"; CFG=c3 STEPS=400 bash tools/ab_bench.sh "base;base" "skew;skew" || exit 1
echo "== c5"; CFG=c5 bash tools/ab_bench.sh "base;base" "skew;skew" || exit 1
