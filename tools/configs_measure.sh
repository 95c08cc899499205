#!/bin/bash
# Bench line of every BASELINE config other than C3 (default warmup/steps, no CPU leg), one box.
# Usage (via gpurun): bash tools/configs_measure.sh <tag>
set -o pipefail
tag=${1:-cfg}
out=gpurun_out/$tag; mkdir -p $out
for c in c2 c4 c5 c5h; do
  timeout -k 10 240 python bench.py --config $c --no-cpu-baseline > $out/bench_$c.json 2> $out/bench_$c.err || { tail -n 20 $out/bench_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out/bench_$c.json'));r=d['chain_roofline'];print('$c',d['value'],d['ms_per_step'],r['tx_ms'],r['rx_ms'],r['chain_ms'],r['frac'],d['decisions_match_sent'])"
done
