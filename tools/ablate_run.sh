#!/bin/bash
# Time every ablation variant (run on the GPU box): kernel-trace stats per variant.
export TMPDIR=/tmp
cfg=${1:-c3}
for v in ${VARIANTS:-base FIR TRIG MIX STORE LOAD}; do
  RUST_MODEM_AMD_LIB=$PWD/rust-modem_amd/build/ablate/$v/libmodem_hip.so timeout -k 10 200 \
    rocprofv3 --kernel-trace --stats -d gpurun_out/abl_$v -o run --output-format csv -- \
    python3 tools/prof_kernels.py --config $cfg --reps 20 > gpurun_out/abl_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
  grep -E "tx_fast|rx_fast|tx_mfma|rx_mfma" gpurun_out/abl_$v/run_kernel_stats.csv | awk -F'",' '{split($2,a,","); printf "   %-45s avg %8.1f us\n", substr($1,2,45), a[3]/1000}'
done
