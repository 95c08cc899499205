#!/bin/bash
# A/B of variant builds (tools/build_var.sh) with the loopback check of each: kernel-trace
# stats per variant + "ok True" when the C3 decisions equal the symbols sent.
export TMPDIR=/tmp
cfg=${CFG:-c3}
for v in "$@"; do
  RUST_MODEM_AMD_LIB=$PWD/rust-modem_amd/build/var/$v/libmodem_hip.so timeout -k 10 60 \
    rocprofv3 --kernel-trace --stats -d gpurun_out/ab_$v -o run --output-format csv -- \
    python3 tools/prof_kernels.py --config $cfg --reps 20 > gpurun_out/ab_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc $(grep -E '^ok' gpurun_out/ab_$v.log)"
  case $rc in 124|134|137|139) exit $rc;; esac
  [ $rc -ne 0 ] && { tail -5 gpurun_out/ab_$v.log; exit $rc; }
  grep -E "tx_fast|rx_fast|tx_mfma|rx_mfma" gpurun_out/ab_$v/run_kernel_stats.csv | awk -F'",' '{split($2,a,","); printf "   %-45s avg %8.1f us  min %8.1f\n", substr($1,2,45), a[3]/1000, a[5]/1000}'
done
