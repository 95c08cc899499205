#!/bin/bash
# A/B kernel timing of alternative library builds under rust-modem_amd/build/var/<name>/
# (run on the GPU box): kernel-trace stats of tools/prof_kernels.py per variant.
export TMPDIR=/tmp
cfg=${CFG:-c3}
for v in "$@"; do
  RUST_MODEM_AMD_LIB=$PWD/rust-modem_amd/build/var/$v/libmodem_hip.so timeout -k 10 200 \
    rocprofv3 --kernel-trace --stats -d gpurun_out/ab_$v -o run --output-format csv -- \
    python3 tools/prof_kernels.py --config $cfg --reps 20 > gpurun_out/ab_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
  grep -E "tx_fast|rx_fast|tx_mfma|rx_mfma" gpurun_out/ab_$v/run_kernel_stats.csv | awk -F'",' '{split($2,a,","); printf "   %-45s avg %8.1f us\n", substr($1,2,45), a[3]/1000}'
done
