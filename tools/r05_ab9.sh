#!/bin/bash
# Round 5 experiment: the TX with a second plane set (MODEM_TX_DBUF: the next tile staged while the
# current one's filter runs, one barrier per tile) against the same DEV_MIN build, C3 and C5.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/r05k; mkdir -p $o
for cfg in c3 c5; do
  CFG=$cfg STEPS=100 timeout -k 10 600 bash tools/ab_bench.sh "$cfg-base;base;" "$cfg-txdb;txdb;" > $o/ab_$cfg.txt 2>&1 || { cat $o/ab_$cfg.txt; exit 1; }
  cat $o/ab_$cfg.txt
done
RUST_MODEM_AMD_LIB=$PWD/rust-modem_amd/build/var/txdb/libmodem_hip.so timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $o/tr -o run -- python3 tools/prof_kernels.py --config c3 --reps 3 > $o/tr.log 2>&1 || exit 1
python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$o/tr/*kernel_trace.csv')[0])):
    if 'tx_mfma' in r['Kernel_Name']: print(r['Kernel_Name'][:60], r.get('VGPR_Count'), r.get('SGPR_Count'), r.get('Scratch_Size'), r.get('LDS_Block_Size', r.get('Lds_Size'))); break"
