#!/bin/bash
# Round 5: how much of the fused small call (C2) is the last workgroup's extra work (the TX tiles
# past the last RX tile + the RX history read)? Timing probe: -DMODEM_CHAIN_NOTAIL skips both
# (wrong history, timing only) against the same-flags base build, alternated three times.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r05ab19}; mkdir -p $o
B="--steps 400 --warmup 100 --settle-ms 200 --no-cpu-baseline --no-out-of-cache"
line() { python3 -c "
import json;d=json.loads([l for l in open('$1') if l.startswith('{')][-1]);c=d['chain_roofline']
print('$2', d['value'], d['ms_per_step'], 'chain', c['chain_ms'])"; }
for rep in 1 2 3; do
  for v in base notail; do
    RUST_MODEM_AMD_LIB=$PWD/rust-modem_amd/build/var/$v/libmodem_hip.so timeout -k 10 300 python3 bench.py --config c2 $B > $o/c2_$v.json 2> $o/err || { tail -3 $o/err; exit 1; }
    line $o/c2_$v.json "c2 $v"
  done
done
