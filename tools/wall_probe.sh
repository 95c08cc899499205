#!/bin/bash
# Wall-clock bench value vs warmup / timed-step counts (C3, one box): shows how long the
# back-to-back launches take to reach their steady rate. Usage (via gpurun): bash tools/wall_probe.sh
set -o pipefail
mkdir -p gpurun_out/wp
for w in 50 2000; do for s in 500 3000; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-out-of-cache --warmup $w --steps $s \
      > gpurun_out/wp/b_${w}_${s}.json 2> gpurun_out/wp/err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/wp/b_${w}_${s}.json'));print($w,$s,d['value'],d['ms_per_step'],d['chain_roofline']['chain_ms'])"
done; done
