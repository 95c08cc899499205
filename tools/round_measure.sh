#!/bin/bash
# The round's evidence pass on one GPU box: parity suite + smoke, three driver-style C3 lines + the
# defaults line, the kernel trace of the driver-style command, C3 PMC passes, every other config's
# line, and PMC traffic for c5 / c5h. Stops at the first failing step.
# Usage (via gpurun): bash tools/round_measure.sh <tag>
set -o pipefail
tag=${1:-r06}
root=${GRAFT_REPO_ROOT:-$(pwd)}
out="$root/gpurun_out/$tag"
mkdir -p "$out"
cd "$root"
echo "[1/6] gpu tests, smoke $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { tail -30 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { tail -20 "$out/smoke.log"; exit 1; }
tail -2 "$out/smoke.log"
echo "[2/6] bench C3: driver style (20 + 5 steps) x3, then defaults $(date +%T)"
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$out/bench_drv$k.json" 2> "$out/bench_drv$k.err" || { tail -20 "$out/bench_drv$k.err"; exit 2; }
  python3 -c "import json;d=json.load(open('$out/bench_drv$k.json'));r=d['roofline'];c=d['chain_roofline'];print('drv$k',d['value'],d['ms_per_step'],r['kernel'],r['frac'],c['tx_ms'],c['rx_ms'],c['chain_ms'],c['frac'],d['decisions_match_sent'])"
done
timeout -k 10 300 python bench.py > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 2; }
cat "$out/bench.json"
echo "[3/6] kernel trace of the driver-style bench command $(date +%T)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
    python3 "$root/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$out/trace.log" 2>&1 || { tail -20 "$out/trace.log"; exit 3; }
cd "$root"
python3 tools/trace_legs.py "$out/trace/run_kernel_trace.csv" > "$out/trace_legs.json"
grep -o '"chain_roofline": {[^}]*}' "$out/trace.log" >> "$out/trace_legs.json" || true
cat "$out/trace_legs.json"
echo "[4/6] pmc c3 $(date +%T)"
bash tools/pmc.sh "$out/pmc" c3 || exit 4
python3 tools/pmc_summary.py "$out/pmc" > "$out/pmc_summary.txt"
echo "[5/6] other configs $(date +%T)"
bash tools/configs_measure.sh "$tag/cfg" || exit 5
echo "[6/6] traffic c5, c5h (FETCH_SIZE, WRITE_SIZE passes) $(date +%T)"
for c in c5 c5h; do
  i=0
  for ctr in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $ctr --output-format csv -d "$out/pmc_$c/p$i" -o run -- python3 tools/prof_kernels.py --config $c --reps 4 > "$out/pmc_$c.$ctr.log" 2>&1 || { tail -5 "$out/pmc_$c.$ctr.log"; exit 6; }
  done
  python3 tools/pmc_summary.py "$out/pmc_$c" > "$out/pmc_$c.txt"
done
echo done $(date +%T)
