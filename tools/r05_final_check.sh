#!/bin/bash
# Round 5: the shipped library after its last rebuild: GPU suite, smoke, three driver-style C3 lines.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
o=gpurun_out/${OUT:-r05fc}; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -n 1 $o/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
tail -n 1 $o/smoke.log
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $o/bench_drv$k.json 2> $o/bench_drv$k.err || { tail -20 $o/bench_drv$k.err; exit 2; }
  python3 -c "import json;d=json.load(open('$o/bench_drv$k.json'));c=d['chain_roofline'];print('drv$k',d['value'],d['ms_per_step'],d['roofline']['frac'],c['chain_ms'],d['decisions_match_sent'])"
done
