#!/bin/bash
# Round 5: the TX staging's LUT reads batched before its plane writes (in-tree) against `kb` (the
# library before it): GPU suite on the tree, then C3, C5, C5 f16, C4, C2, alternated twice.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r05t}; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.txt 2>&1 || { tail -20 $o/gpu_tests.txt; exit 1; }
tail -2 $o/gpu_tests.txt
B="--steps 200 --warmup 50 --settle-ms 200 --no-cpu-baseline --no-out-of-cache"
line() { python3 -c "
import json;d=json.loads([l for l in open('$1') if l.startswith('{')][-1]);c=d['chain_roofline']
print('$2', d['value'], d['ms_per_step'], 'tx', c['tx_ms'], 'rx', c['rx_ms'], 'chain', c['chain_ms'], d['decisions_match_sent'])"; }
for rep in 1 2; do
  for cfg in c3 c5 c5h c4 c2; do
    for v in kb tree; do
      lib=""; [ $v != tree ] && lib="$PWD/rust-modem_amd/build/var/$v/libmodem_hip.so"
      RUST_MODEM_AMD_LIB=$lib timeout -k 10 300 python3 bench.py --config $cfg $B > $o/${cfg}_$v.json 2> $o/err || { tail -3 $o/err; exit 1; }
      line $o/${cfg}_$v.json "$cfg $v"
    done
  done
done
