#!/bin/bash
# Interleaved bench A/B of two tools/build_var.sh builds (base, prio) on one box: the default
# C3 bench line per run, without the CPU and out-of-cache legs. Usage (via gpurun): bash tools/wall_ab.sh
for i in 1 2 3; do
 for v in base prio; do
  RUST_MODEM_AMD_LIB=$PWD/rust-modem_amd/build/var/$v/libmodem_hip.so timeout -k 10 120 python bench.py --no-cpu-baseline --no-out-of-cache > gpurun_out/wb_$v$i.json 2>gpurun_out/wb_$v$i.err || exit $?
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/wb_$v$i.json') if l.startswith('{')][0]); print('$v$i', d['value'], d['ms_per_step'], d['chain_roofline']['tx_ms'], d['chain_roofline']['rx_ms'], d['decisions_match_sent'])"
 done
done
