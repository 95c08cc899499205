#!/bin/bash
# Round 5: wide TX tiles at sps 8 (MODEM_TX_WIDE build) on C5 f16 and f32; kernel traces of the
# 4-channel batch probes (which kernels, their durations and register counts).
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/r05c; mkdir -p $o
for cfg in c5h c5; do
  CFG=$cfg STEPS=30 timeout -k 10 600 bash tools/ab_bench.sh "$cfg-base;;" "$cfg-wide;wide;" > $o/ab_$cfg.txt 2>&1 || { cat $o/ab_$cfg.txt; exit 1; }
  cat $o/ab_$cfg.txt
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_q16b -o run -- python3 tools/wl_probe.py qam16 4 129 4 4194304 4 > $o/tr_q16b.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_qpb -o run -- python3 tools/wl_probe.py qpsk 2 65 4 4194304 4 > $o/tr_qpb.log 2>&1 || exit $?
RUST_MODEM_AMD_LIB=$PWD/rust-modem_amd/build/var/wide/libmodem_hip.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_wide -o run -- python3 tools/prof_kernels.py --config c5h --reps 3 > $o/tr_wide.log 2>&1 || exit $?
grep -h '"label"' $o/tr_*.log
