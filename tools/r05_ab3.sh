#!/bin/bash
# Round 5: C4 job step forms (MODEM_BENCH_BATCH) at groups of 8 and 4; C5 f16 RX with the taps'
# f16 roundings only (build/var/nolo: -DMODEM_RX_HI_NOLO=1) against the tree, and its error.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/r05e; mkdir -p $o
B="--steps 200 --warmup 50 --settle-ms 200 --no-cpu-baseline --no-out-of-cache"
for rep in 1 2; do
  for g in 8 4; do
    for mode in cbp plans streams2; do
      MODEM_BENCH_BATCH=$mode timeout -k 10 300 python3 bench.py --config c4 --group $g $B > $o/c4_${mode}_g${g}_$rep.json 2> $o/c4.err || { tail -3 $o/c4.err; exit 1; }
      python3 -c "
import json;d=json.loads([l for l in open('$o/c4_${mode}_g${g}_$rep.json') if l.startswith('{')][-1])
print('c4 $mode g$g', d['value'], d['ms_per_step'], d['decisions_match_sent'])"
    done
  done
done
CFG=c5h STEPS=30 timeout -k 10 600 bash tools/ab_bench.sh "c5h-base;;" "c5h-nolo;nolo;" > $o/ab_nolo.txt 2>&1 || { cat $o/ab_nolo.txt; exit 1; }
cat $o/ab_nolo.txt
RUST_MODEM_AMD_LIB=$PWD/rust-modem_amd/build/var/nolo/libmodem_hip.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_range.py -q -s -k "c5_prefix or f16_large" --timeout 200 --timeout-method thread > $o/nolo_err.log 2>&1
grep "range\]" $o/nolo_err.log; tail -2 $o/nolo_err.log
