#!/bin/bash
# A/B of environment settings on the in-tree library: kernel-trace stats per setting + the
# C3 loopback check. Usage: tools/ab_env.sh "VAR=val ..." "" ...  ("" = defaults)
export TMPDIR=/tmp
cfg=${CFG:-c3}
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 60 rocprofv3 --kernel-trace --stats -d gpurun_out/abe_$i -o run --output-format csv -- \
    python3 tools/prof_kernels.py --config $cfg --reps 20 > gpurun_out/abe_$i.log 2>&1
  rc=$?
  echo "== [$e] rc=$rc $(grep -E '^ok' gpurun_out/abe_$i.log)"
  case $rc in 124|134|137|139) exit $rc;; esac
  [ $rc -ne 0 ] && { tail -5 gpurun_out/abe_$i.log; exit $rc; }
  grep -E "tx_mfma|rx_mfma" gpurun_out/abe_$i/run_kernel_stats.csv | awk -F'",' '{split($2,a,","); printf "   %-45s avg %8.1f us  min %8.1f\n", substr($1,2,45), a[3]/1000, a[5]/1000}'
done
