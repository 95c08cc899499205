#!/bin/bash
# Round 5: the RX filter's double-buffered operands (MODEM_RX_DB) and late slot reloads
# (MODEM_RX_LATE) re-measured now that the staging waits are exact (DEV_MIN builds, C3, twice);
# then three driver-style C3 lines of the in-tree library.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r05n}; mkdir -p $o
B="--steps 200 --warmup 50 --settle-ms 200 --no-cpu-baseline --no-out-of-cache"
line() { python3 -c "
import json;d=json.loads([l for l in open('$1') if l.startswith('{')][-1]);c=d['chain_roofline']
print('$2', d['value'], d['ms_per_step'], 'tx', c['tx_ms'], 'rx', c['rx_ms'], 'chain', c['chain_ms'], d['decisions_match_sent'])"; }
for rep in 1 2; do
  for v in dm0 dmdb dmlate; do
    RUST_MODEM_AMD_LIB=$PWD/rust-modem_amd/build/var/$v/libmodem_hip.so timeout -k 10 300 python3 bench.py --config c3 $B > $o/c3_$v.json 2> $o/err || { tail -3 $o/err; exit 1; }
    line $o/c3_$v.json "c3 $v"
  done
done
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $o/c3_drv$i.json 2> $o/err || { tail -3 $o/err; exit 1; }
  line $o/c3_drv$i.json "c3 driver-style $i"
done
