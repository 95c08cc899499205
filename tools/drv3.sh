#!/bin/bash
# GPU tests, then three driver-style C3 bench lines (--steps 20 --warmup 5) and one with defaults.
# Usage (via gpurun): bash tools/drv3.sh <tag> [skip-tests]
set -o pipefail
tag=${1:-r03c}; root=${GRAFT_REPO_ROOT:-$(pwd)}; out="$root/gpurun_out/$tag"; mkdir -p "$out"; cd "$root"
if [ -z "$2" ]; then
  echo "[tests]"
  timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { tail -30 "$out/gpu_tests.log"; exit 1; }
  tail -1 "$out/gpu_tests.log"
fi
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-out-of-cache > "$out/bench_drv$k.json" 2> "$out/bench_drv$k.err" || { tail -20 "$out/bench_drv$k.err"; exit 2; }
  python3 -c "import json;d=json.load(open('$out/bench_drv$k.json'));r=d['roofline'];c=d['chain_roofline'];print('drv$k',d['value'],d['ms_per_step'],r['kernel'],r['frac'],c['tx_ms'],c['rx_ms'],c['chain_ms'],c['frac'],d['decisions_match_sent'])"
done
timeout -k 10 300 python bench.py --no-cpu-baseline > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 2; }
cat "$out/bench.json"
