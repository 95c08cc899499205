#!/bin/bash
# Round 6's GPU-box probes in one place (measurement tooling; each writes under gpurun_out/$OUT and
# stops at the first failing step). Library variants for A/B runs: tools/build_var.sh + tools/ab_variants.sh.
# Usage (via gpurun): [OUT=dir] [LIB=path/to/libmodem_hip.so] bash tools/probes.sh <probe>
#   c4-layout   C4 batch legs vs the placement of the channels' sample buffers (tools/c4_layout_probe.py)
#   c4-batch    the batch launches against one channel: 1 x 2^24, the batch kernel on 1 x 2^24, 2 x 2^23,
#               4 x 2^22, 8 x 2^21 QPSK, C3 single vs batch-of-one (tools/wl_probe.py)
#   c4-rot      the batch's per-channel workgroup rotation, MODEM_BATCH_ROT=0 vs 1, probes and the job
#   c4-groups   the C4 job's group size (8, 4, 2) and TX store policy (MODEM_TX_NT=0)
#   c2-legs     C2's legs and fused launch (tools/wl_probe.py), three times
#   scan        the scanned phasors: tests/test_stateful.py, then tools/scan_rate.py under a kernel trace
#   store-cal   buffer-store range checks (tools/ubench/oob_store) and WRITE_SIZE per store pattern
#               (tools/ubench/write_cal under rocprofv3 --pmc WRITE_SIZE)
#   c5h-writes  C5 f16 RX WRITE_SIZE (one rocprofv3 --pmc pass over tools/prof_kernels.py --only rx)
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/${OUT:-probe}; mkdir -p $o
[ -n "$LIB" ] && export RUST_MODEM_AMD_LIB=$LIB
wl() { timeout -k 10 150 python3 tools/wl_probe.py "$@" >> $o/probe.txt 2>> $o/err || { tail -5 $o/err; exit 1; }; tail -1 $o/probe.txt; }
case "$1" in
c4-layout)
  wl qpsk 2 65 4 16777216 1 --label single24
  for a in "--group 4 --separate" "--group 4 --stagger 0" "--group 4 --stagger 4096" "--group 4 --stagger 266240" \
           "--group 8 --separate" "--group 8 --stagger 0" "--group 8 --stagger 4096"; do
    timeout -k 10 150 python3 tools/c4_layout_probe.py $a >> $o/probe.txt 2>> $o/err || { tail -5 $o/err; exit 1; }
    tail -1 $o/probe.txt
  done ;;
c4-batch)
  wl qpsk 2 65 4 16777216 1 --label single24; wl qpsk 2 65 4 16777216 1 --batch --label batch1x24
  wl qpsk 2 65 4 4194304 1 --label single22; wl qpsk 2 65 4 8388608 2 --label batch2x23
  wl qpsk 2 65 4 4194304 4 --label batch4x22; wl qpsk 2 65 4 2097152 8 --label batch8x21
  wl qam16 4 129 4 16777216 1 --batch --label c3batch1; wl qam16 4 129 4 16777216 1 --label c3single ;;
c4-rot)
  for rep in 1 2; do for rot in 0 1; do
    MODEM_BATCH_ROT=$rot wl qpsk 2 65 4 4194304 4 --label batch4x22_rot$rot
    MODEM_BATCH_ROT=$rot wl qpsk 2 65 4 2097152 8 --label batch8x21_rot$rot
  done; done
  OUT=${OUT:-probe}/ab VARIANTS="tree:MODEM_BATCH_ROT=0 tree" CONFIGS="c4" REPS=2 bash tools/ab_variants.sh ;;
c4-groups)
  B="--steps 100 --warmup 30 --settle-ms 200 --no-cpu-baseline --no-out-of-cache"
  for rep in 1 2; do for v in "8:2" "4:2" "8:0" "2:2"; do
    g=${v%%:*}; nt=${v#*:}
    MODEM_TX_NT=$nt timeout -k 10 300 python3 bench.py --config c4 --group $g $B > $o/c4_g${g}_nt$nt.json 2> $o/err || { tail -3 $o/err; exit 1; }
    python3 -c "
import json;d=json.loads([l for l in open('$o/c4_g${g}_nt$nt.json') if l.startswith('{')][-1]);c=d['chain_roofline']
print('c4 group $g MODEM_TX_NT=$nt', d['value'], d['ms_per_step'], round(d['value']*18.75/8000/1000,4), 'tx', c['tx_ms'], 'rx', c['rx_ms'], 'chain', c['chain_ms'], d['decisions_match_sent'])" | tee -a $o/lines.txt
  done; done ;;
c2-legs)
  for rep in 1 2 3; do wl qpsk 2 65 4 1048576 1 --label c2; done ;;
scan)
  timeout -k 10 300 python3 -u -m pytest tests/test_stateful.py -x -q --timeout 200 --timeout-method thread > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
  tail -1 $o/tests.txt
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/scan_trace -o run -- python3 tools/scan_rate.py > $o/scan_rate.txt 2>&1 || { tail -20 $o/scan_rate.txt; exit 1; }
  grep phasor $o/scan_rate.txt
  grep -h "tx_scan" $o/scan_trace/*kernel_stats.csv | cut -c1-160 ;;
store-cal)
  timeout -k 5 60 tools/ubench/oob_store > $o/oob_store.txt 2>&1 || { cat $o/oob_store.txt; exit 1; }
  cat $o/oob_store.txt
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/wcal -o run -- tools/ubench/write_cal > $o/wcal.log 2>&1 || { tail -5 $o/wcal.log; exit 1; }
  python3 tools/pmc_summary.py $o/wcal ;;
c5h-writes)
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/pmc_w/p1 -o run -- python3 tools/prof_kernels.py --config c5h --reps 4 --only rx > $o/pmc_w.log 2>&1 || { tail -5 $o/pmc_w.log; exit 1; }
  python3 tools/pmc_summary.py $o/pmc_w | grep -A1 rx_mfma ;;
*)
  sed -n '2,18p' "$0"; exit 2 ;;
esac
