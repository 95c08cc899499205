#!/bin/bash
# Round 5: the chain batch's two lanes (C4 job) and pipelined periods (MODEM_BENCH_PIPE) on the
# one-channel configs, each against its one-stream form, alternated twice.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/r05f; mkdir -p $o
B="--steps 200 --warmup 50 --settle-ms 200 --no-cpu-baseline --no-out-of-cache"
line() { python3 -c "
import json;d=json.loads([l for l in open('$1') if l.startswith('{')][-1]);c=d['chain_roofline']
print('$2', d['value'], d['ms_per_step'], 'chain', c['chain_ms'], d['decisions_match_sent'])"; }
for rep in 1 2; do
  for g in 8; do
    for lanes in 2; do
      MODEM_CHAIN_BATCH_LANES=$lanes timeout -k 10 300 python3 bench.py --config c4 --group $g $B > $o/c4_g${g}_l$lanes.json 2> $o/err || { tail -3 $o/err; exit 1; }
      line $o/c4_g${g}_l$lanes.json "c4 g$g lanes$lanes"
    done
  done
  for cfg in c3 c5 c5h; do
    for pipe in 0 1; do
      MODEM_BENCH_PIPE=$pipe timeout -k 10 300 python3 bench.py --config $cfg $B > $o/${cfg}_p$pipe.json 2> $o/err || { tail -3 $o/err; exit 1; }
      line $o/${cfg}_p$pipe.json "$cfg pipe$pipe"
    done
  done
  MODEM_BENCH_PIPE=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-out-of-cache > $o/c3_p1_drv.json 2> $o/err || exit 1
  line $o/c3_p1_drv.json "c3 pipe1 driver-style"
done
