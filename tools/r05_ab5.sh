#!/bin/bash
# Round 5: what the call's first RX tile (the general path: its window reads the history) costs
# at the kernel's end: every tile on the fast path (-DMODEM_RX_NOGEN, wrong results by design:
# the first tile's history samples stage as zeros) against the same DEV_MIN build.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/r05g; mkdir -p $o
for cfg in c3 c5; do
  CFG=$cfg STEPS=100 timeout -k 10 600 bash tools/ab_bench.sh "$cfg-base;base;" "$cfg-nogen;nogen;" > $o/ab_$cfg.txt 2>&1 || { cat $o/ab_$cfg.txt; exit 1; }
  cat $o/ab_$cfg.txt
done
