#!/bin/bash
# One GPU-box pass for the round's evidence: parity suite, default bench line, kernel-trace
# stats of the bench command, PMC traffic passes. Stops at the first failing step.
# Usage (via gpurun): bash tools/round_measure.sh <tag>
set -o pipefail
tag=${1:-r01}
root=${GRAFT_REPO_ROOT:-$(pwd)}
out="$root/gpurun_out/$tag"
mkdir -p "$out"
cd "$root"
echo "[1/4] gpu tests"
timeout -k 10 420 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { tail -30 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
echo "[2/4] bench"
timeout -k 10 300 python bench.py > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 2; }
cat "$out/bench.json"
echo "[3/4] kernel trace"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
    python3 "$root/bench.py" --no-cpu-baseline > "$out/trace.log" 2>&1 || { tail -20 "$out/trace.log"; exit 3; }
cd "$root"
python3 tools/trace_legs.py "$out/trace/run_kernel_trace.csv" > "$out/trace_legs.json"
grep -o '"chain_roofline": {[^}]*}' "$out/trace.log" >> "$out/trace_legs.json" || true
cat "$out/trace_legs.json"
echo "[4/4] pmc"
bash tools/pmc.sh "$out/pmc" c3 || exit 4
python3 tools/pmc_summary.py "$out/pmc" > "$out/pmc_summary.txt"
echo done
