#!/bin/bash
# Round 5: the C4 job with a per-lane ring of sample buffers (MODEM_BENCH_RING=1: the samples of
# group k land in lane k % 2's slots, so they stay in the Infinity Cache between the TX and the
# RX) against one buffer per channel, groups of 2, 4 and 8, alternated twice; then the
# chain-batch tests (new lanes test) and three driver-style C3 lines with the 500 ms settle.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/r05g; mkdir -p $o
B="--steps 200 --warmup 50 --settle-ms 200 --no-cpu-baseline --no-out-of-cache"
line() { python3 -c "
import json;d=json.loads([l for l in open('$1') if l.startswith('{')][-1]);c=d['chain_roofline']
print('$2', d['value'], d['ms_per_step'], 'chain', c['chain_ms'], d['decisions_match_sent'], d['roofline']['frac'])"; }
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_chain_batch.py > $o/tests.txt 2>&1 || { tail -5 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
for rep in 1 2; do
  for g in 2 4 8; do
    for ring in 0 1; do
      MODEM_BENCH_RING=$ring timeout -k 10 300 python3 bench.py --config c4 --group $g $B > $o/c4_g${g}_r$ring.json 2> $o/err || { tail -3 $o/err; exit 1; }
      line $o/c4_g${g}_r$ring.json "c4 g$g ring$ring"
    done
  done
done
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $o/c3_drv$i.json 2> $o/err || { tail -3 $o/err; exit 1; }
  line $o/c3_drv$i.json "c3 driver-style $i"
done
