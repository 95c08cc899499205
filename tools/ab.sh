#!/bin/bash
# A/B on the GPU box: kernel-trace stats of tools/prof_kernels.py (with its poisoned-output
# loopback check) for each case "label;ENV=val ...;variant" (variant: a tools/build_var.sh
# build under rust-modem_amd/build/var/, empty = the in-tree library). Extra prof_kernels
# arguments via PK (e.g. PK="--amplitude 0.0625"); config via CFG.
export TMPDIR=/tmp
cfg=${CFG:-c3}
for c in "$@"; do
  IFS=';' read -r label envs var <<< "$c"
  lib=""; [ -n "$var" ] && lib="RUST_MODEM_AMD_LIB=$PWD/rust-modem_amd/build/var/$var/libmodem_hip.so"
  env $envs $lib timeout -k 10 90 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_$label -o run --output-format csv -- \
    python3 tools/prof_kernels.py --config $cfg --reps ${REPS:-20} $PK > gpurun_out/ab_$label.log 2>&1
  rc=$?
  echo "== $label [$envs] [$var] rc=$rc $(grep -E '^ok' gpurun_out/ab_$label.log)"
  case $rc in 124|134|137|139) exit $rc;; esac
  [ $rc -ne 0 ] && { tail -5 gpurun_out/ab_$label.log; exit $rc; }
  grep -E "tx_mfma|rx_mfma|rx_ring|tx_fast|chain_mfma" gpurun_out/ab_$label/run_kernel_stats.csv | awk -F'",' '{split($2,a,","); printf "   %-40s n %5d avg %8.2f us  min %8.2f\n", substr($1,2,40), a[1], a[3]/1000, a[5]/1000}'
done
