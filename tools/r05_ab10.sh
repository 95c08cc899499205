#!/bin/bash
# Round 5: TX held to 4 waves per SIMD (MODEM_TX_WPE=4: C5 f32's TX 132 -> 125 VGPRs, 3 -> 4 waves)
# and the B-fragment pin (nopin: MODEM_TX_PIN_B=0) against the in-tree library, alternated twice.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/r05l; mkdir -p $o
B="--steps 200 --warmup 50 --settle-ms 200 --no-cpu-baseline --no-out-of-cache"
line() { python3 -c "
import json;d=json.loads([l for l in open('$1') if l.startswith('{')][-1]);c=d['chain_roofline']
print('$2', d['value'], d['ms_per_step'], 'tx', c['tx_ms'], 'rx', c['rx_ms'], 'chain', c['chain_ms'], d['decisions_match_sent'])"; }
for rep in 1 2; do
  for cfg in c5 c3 c5h c4; do
    for v in tree wpe4 nopin; do
      lib=""; [ $v != tree ] && lib="$PWD/rust-modem_amd/build/var/$v/libmodem_hip.so"
      RUST_MODEM_AMD_LIB=$lib timeout -k 10 300 python3 bench.py --config $cfg $B > $o/${cfg}_$v.json 2> $o/err || { tail -3 $o/err; exit 1; }
      line $o/${cfg}_$v.json "$cfg $v"
    done
  done
done
