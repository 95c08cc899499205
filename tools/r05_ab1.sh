#!/bin/bash
# Round 5: RX LATE/DB variants on C3 (tools/ab_bench.sh) and the batch-vs-single-channel probe.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/r05b; mkdir -p $o
CFG=c3 timeout -k 10 600 bash tools/ab_bench.sh "base;base;" "l2d1;l2d1;" "l1d1;l1d1;" "l2d0;l2d0;" > $o/ab_rx.txt 2>&1 || { cat $o/ab_rx.txt; exit 1; }
cat $o/ab_rx.txt
for w in "qam16 4 129 4 16777216 1" "qpsk 2 65 4 16777216 1" "qpsk 2 65 4 4194304 4" "qam16 4 129 4 4194304 4" "qpsk 2 65 4 4194304 4 0 --no-batch"; do
  timeout -k 10 120 python3 tools/wl_probe.py $w >> $o/wl.txt 2>> $o/wl.err || { tail -5 $o/wl.err; exit 1; }
done
cat $o/wl.txt
