#!/bin/bash
# Round 5: GPU suite on the tree (wide TX at sps 8, modem_chain_batch), then bench lines.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/r05d; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1
rc=$?; tail -3 $o/gpu_tests.log; [ $rc = 0 ] || exit $rc
B="--steps 200 --warmup 50 --no-cpu-baseline --no-out-of-cache"
for c in "c4 --group 8" "c4 --group 4" "c5" "c5h"; do
  n=$(echo $c | tr -d ' -')
  timeout -k 10 300 python3 bench.py --config $c $B > $o/b_$n.json 2> $o/b_$n.err || { tail -3 $o/b_$n.err; exit 1; }
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $o/b_c3drv.json 2> $o/b_c3drv.err || exit 1
for f in $o/b_*.json; do python3 -c "
import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);c=d['chain_roofline'];r=d['roofline']
print('$f', d['value'], 'ms/step',d['ms_per_step'],'tx',c['tx_ms'],'rx',c['rx_ms'],'chain',c['chain_ms'],'chain_frac',c['frac'],'dom',r['frac'],'traffic',r['traffic'],'ok',d['decisions_match_sent'], d.get('roofline_out_of_cache',{}).get('frac'))"; done
