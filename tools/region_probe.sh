#!/bin/bash
# tools/region_probe.py under several preambles, one box. Usage (via gpurun): bash tools/region_probe.sh <tag>
set -o pipefail
tag=${1:-probe}; root=${GRAFT_REPO_ROOT:-$(pwd)}; out="$root/gpurun_out/$tag"; mkdir -p "$out"; cd "$root"
for pre in settle none settle w2000; do
  timeout -k 10 120 python tools/region_probe.py --preamble $pre >> "$out/probe.txt" 2>&1 || exit 1
done

cat "$out/probe.txt"
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-out-of-cache > "$out/bench_drv$k.json" 2> "$out/bench_drv$k.err" || { tail -20 "$out/bench_drv$k.err"; exit 2; }
  python3 -c "import json;d=json.load(open('$out/bench_drv$k.json'));r=d['roofline'];c=d['chain_roofline'];print('drv$k',d['value'],d['ms_per_step'],r['kernel'],r['frac'],c['tx_ms'],c['rx_ms'],c['chain_ms'],c['frac'],d['decisions_match_sent'],d['settle'])"
done
