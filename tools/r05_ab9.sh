#!/bin/bash
# Round 5: the two parts of the store change apart (DEV_MIN builds, f32 configs): g = sample stores
# through global pointers (else generic / flat), p = TX B fragments pinned at the kernel's start.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/r05j; mkdir -p $o
B="--steps 200 --warmup 50 --settle-ms 200 --no-cpu-baseline --no-out-of-cache"
line() { python3 -c "
import json;d=json.loads([l for l in open('$1') if l.startswith('{')][-1]);c=d['chain_roofline']
print('$2', d['value'], d['ms_per_step'], 'tx', c['tx_ms'], 'rx', c['rx_ms'], 'chain', c['chain_ms'], d['decisions_match_sent'])"; }
for rep in 1 2; do
  for cfg in c3 c4 c5; do
    for v in g0p0 g1p0 g0p1 g1p1; do
      RUST_MODEM_AMD_LIB=$PWD/rust-modem_amd/build/var/$v/libmodem_hip.so timeout -k 10 300 python3 bench.py --config $cfg $B > $o/${cfg}_$v.json 2> $o/err || { tail -3 $o/err; exit 1; }
      line $o/${cfg}_$v.json "$cfg $v"
    done
  done
done
