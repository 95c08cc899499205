#!/bin/bash
# Round 5: the C4 job's TX store policy: MODEM_TX_NT=0 (no non-temporal stores) against the default
# (a batch launch over 192 MiB stores all its samples non-temporally), groups of 8, three alternations.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r05q}; mkdir -p $o
B="--steps 100 --warmup 30 --settle-ms 200 --no-cpu-baseline --no-out-of-cache"
for rep in 1 2 3; do
  for nt in 2 0; do
    MODEM_TX_NT=$nt timeout -k 10 300 python3 bench.py --config c4 $B > $o/c4_nt$nt.json 2> $o/err || { tail -3 $o/err; exit 1; }
    python3 -c "
import json;d=json.loads([l for l in open('$o/c4_nt$nt.json') if l.startswith('{')][-1]);c=d['chain_roofline']
print('c4 MODEM_TX_NT=$nt', d['value'], d['ms_per_step'], round(d['value']*18.75/8000/1000,4), 'tx', c['tx_ms'], 'rx', c['rx_ms'], d['decisions_match_sent'])"
  done
done
