#!/bin/bash
# Round 5: a one-channel period split into k chunks on two lanes (MODEM_CHAIN_SPLIT=k: chunk i's
# RX beside chunk i+1's TX, same buffers, same results) against the two launches; bench lines.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/r05i; mkdir -p $o
B="--steps 200 --warmup 50 --settle-ms 200 --no-cpu-baseline --no-out-of-cache"
line() { python3 -c "
import json;d=json.loads([l for l in open('$1') if l.startswith('{')][-1]);c=d['chain_roofline']
print('$2', d['value'], d['ms_per_step'], 'chain', c['chain_ms'], 'tx', c['tx_ms'], 'rx', c['rx_ms'], d['decisions_match_sent'])"; }
for rep in 1 2; do
  for cfg in c3 c5 c5h; do
    for k in 1 2 4; do
      MODEM_CHAIN_SPLIT=$k timeout -k 10 300 python3 bench.py --config $cfg $B > $o/${cfg}_k$k.json 2> $o/err || { tail -3 $o/err; exit 1; }
      line $o/${cfg}_k$k.json "$cfg split$k"
    done
  done
done
