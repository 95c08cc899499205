#!/bin/bash
# Round 5: the C4 job's group size (channels per TX / RX launch pair, two lanes) 4 / 8 / 16 / 32, twice.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r05p}; mkdir -p $o
B="--steps 100 --warmup 30 --settle-ms 200 --no-cpu-baseline --no-out-of-cache"
for rep in 1 2; do
  for g in 4 8 16 32; do
    timeout -k 10 300 python3 bench.py --config c4 --group $g $B > $o/c4_g$g.json 2> $o/err || { tail -3 $o/err; exit 1; }
    python3 -c "
import json;d=json.loads([l for l in open('$o/c4_g$g.json') if l.startswith('{')][-1])
print('c4 group $g', d['value'], d['ms_per_step'], round(d['value']*18.75/8000/1000,4), d['decisions_match_sent'])"
  done
done
