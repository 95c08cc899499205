#!/bin/bash
# A/B: ascending RX tile rounds at decim 8 (-DMODEM_RX_ASC) against the base build; C3 with the
# base build against the in-tree library.
cd ${GRAFT_REPO_ROOT:-.}
echo "== c5"; CFG=c5 bash tools/ab_bench.sh "base;base" "asc;asc" || exit 1
echo "== c3"; CFG=c3 STEPS=400 bash tools/ab_bench.sh "tree;;" "base;base" || exit 1
