#!/bin/bash
# Round 5 experiment: consecutive periods pipelined at the C level (MODEM_CHAIN_PIPE=1: odd periods
# into a second sample buffer, each RX on the plan's own stream beside the next period's TX)
# against the one-stream chain; bench lines, two alternations.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/r05j; mkdir -p $o
B="--steps 200 --warmup 50 --settle-ms 200 --no-cpu-baseline --no-out-of-cache"
line() { python3 -c "
import json;d=json.loads([l for l in open('$1') if l.startswith('{')][-1]);c=d['chain_roofline']
print('$2', d['value'], d['ms_per_step'], 'chain', c['chain_ms'], 'tx', c['tx_ms'], 'rx', c['rx_ms'], d['decisions_match_sent'])"; }
for rep in 1 2; do
  for cfg in c3 c5 c5h; do
    for pipe in 0 1; do
      MODEM_CHAIN_PIPE=$pipe timeout -k 10 300 python3 bench.py --config $cfg $B > $o/${cfg}_p$pipe.json 2> $o/err || { tail -3 $o/err; exit 1; }
      line $o/${cfg}_p$pipe.json "$cfg pipe$pipe"
    done
  done
done
MODEM_CHAIN_PIPE=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-out-of-cache > $o/c3_p1_drv.json 2> $o/err || exit 1
line $o/c3_p1_drv.json "c3 pipe1 driver-style"
