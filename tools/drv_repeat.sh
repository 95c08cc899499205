#!/bin/bash
# Driver-style C3 bench lines (--steps 20 --warmup 5, as the round-end driver runs bench.py),
# three in a row on one box. Usage (via gpurun): bash tools/drv_repeat.sh <tag>
set -o pipefail
tag=${1:-drv}; root=${GRAFT_REPO_ROOT:-$(pwd)}; out="$root/gpurun_out/$tag"; mkdir -p "$out"; cd "$root"
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$out/bench_drv$k.json" 2> "$out/bench_drv$k.err" || { tail -20 "$out/bench_drv$k.err"; exit 2; }
  python3 -c "import json;d=json.load(open('$out/bench_drv$k.json'));r=d['roofline'];c=d['chain_roofline'];print('drv$k',d['value'],d['ms_per_step'],r['kernel'],r['frac'],c['tx_ms'],c['rx_ms'],c['chain_ms'],c['frac'],d['decisions_match_sent'],d['roofline_out_of_cache']['chain_frac'],d['cpu_baseline']['value'])"
done
