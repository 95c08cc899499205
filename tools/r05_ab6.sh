#!/bin/bash
# Round 5: C2's byte-pattern floor and empty-launch floor (tools/ubench/chain_floor c2); the RX
# filter double-buffered (MODEM_RX_LATE=1 MODEM_RX_DB=1, build/var/db1) on C5 f16 (20 k-steps),
# C4 and C3 against the tree.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/r05h; mkdir -p $o
timeout -k 10 120 tools/ubench/chain_floor c2 > $o/floor_c2.txt 2>&1 || exit $?
cat $o/floor_c2.txt
for cfg in c5h c4 c3; do
  CFG=$cfg STEPS=50 timeout -k 10 600 bash tools/ab_bench.sh "$cfg-base;;" "$cfg-db1;db1;" > $o/ab_$cfg.txt 2>&1 || { cat $o/ab_$cfg.txt; exit 1; }
  cat $o/ab_$cfg.txt
done
