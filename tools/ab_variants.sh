#!/bin/bash
# A/B of library builds and environment switches by bench.py lines, alternated on one box (the
# parameterised form of round 5's one-off A/B scripts). Usage (via gpurun):
#   OUT=r06x VARIANTS="tree var1 tree:MODEM_TX_NT=0" CONFIGS="c3 c5" REPS=2 [TESTS=1] [DRV=3] \
#     [BENCH="--steps 200 --warmup 50 --settle-ms 200"] bash tools/ab_variants.sh
# A variant is "<lib>[:ENV=val,ENV=val]": lib "tree" = the in-tree library, any other name =
# rust-modem_amd/build/var/<name>/libmodem_hip.so (tools/build_var.sh). TESTS=1 runs the GPU suite on
# the tree first; DRV=n adds n driver-style C3 lines (--steps 20 --warmup 5) of the tree at the end.
# Each line: variant, config, Gs/s, ms per step, the TX / RX / chain legs (HIP events), decisions ok.
# Stops at the first failing step.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/${OUT:-ab}; mkdir -p $o
B=${BENCH:-"--steps 200 --warmup 50 --settle-ms 200"}
B="$B --no-cpu-baseline --no-out-of-cache"
line() { python3 -c "
import json;d=json.loads([l for l in open('$1') if l.startswith('{')][-1]);c=d['chain_roofline']
print('$2', d['value'], d['ms_per_step'], 'tx', c['tx_ms'], 'rx', c['rx_ms'], 'chain', c['chain_ms'], d['decisions_match_sent'])"; }
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.txt 2>&1 || { tail -20 $o/gpu_tests.txt; exit 1; }
  tail -1 $o/gpu_tests.txt
fi
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in ${CONFIGS:-c3}; do
    for v in ${VARIANTS:-tree}; do
      lib=${v%%:*}; envs=""; [ "$lib" != "$v" ] && envs=$(echo "${v#*:}" | tr ',' ' ')
      path=""; [ "$lib" != tree ] && path="$PWD/rust-modem_amd/build/var/$lib/libmodem_hip.so"
      tag=$(echo "${cfg}_$v" | tr ':=,' '___')
      env $envs RUST_MODEM_AMD_LIB=$path timeout -k 10 300 python3 bench.py --config $cfg $B > $o/$tag.json 2> $o/$tag.err || { tail -3 $o/$tag.err; exit 1; }
      line $o/$tag.json "$cfg $v" | tee -a $o/lines.txt
    done
  done
done
for i in $(seq 1 ${DRV:-0}); do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $o/c3_drv$i.json 2> $o/c3_drv$i.err || { tail -3 $o/c3_drv$i.err; exit 1; }
  line $o/c3_drv$i.json "c3 driver-style $i" | tee -a $o/lines.txt
done
