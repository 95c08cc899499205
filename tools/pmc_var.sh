#!/bin/bash
# One PMC pass per variant build (tools/build_var.sh) over the C3 prof workload.
# Usage: tools/pmc_var.sh "<counters>" <variant>...
export TMPDIR=/tmp
ctr=$1; shift
for v in "$@"; do
  RUST_MODEM_AMD_LIB=$PWD/rust-modem_amd/build/var/$v/libmodem_hip.so timeout -s KILL 60 \
    rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmcv_$v -o run -- \
    python3 tools/prof_kernels.py --config c3 --reps 10 > gpurun_out/pmcv_$v.log 2>&1 || exit $?
  echo "== $v"
  python3 - "$v" <<'PY'
import csv, sys, collections
v = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f"gpurun_out/pmcv_{v}/run_counter_collection.csv")):
    k = r["Kernel_Name"]
    if "rx_mfma" in k or "tx_mfma" in k:
        acc[k[:20]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print("  ", k, {c: round(sum(x) / len(x)) for c, x in d.items()})
PY
done
