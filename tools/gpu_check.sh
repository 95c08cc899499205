#!/bin/bash
# GPU-box check: parity suite, then a kernel-trace profile of the bench workload's TX/RX.
# Usage (via gpurun): bash tools/gpu_check.sh <profile-dir-name> [prof_kernels args...]
set -o pipefail
name=${1:-prof}; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$root/gpurun_out"
timeout -k 10 300 python -m pytest "$root/tests" -m gpu -q -x > "$root/gpurun_out/gpu_tests.log" 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$root/gpurun_out/$name" -o run -- \
    python3 "$root/tools/prof_kernels.py" --reps 20 "$@" > "$root/gpurun_out/prof.log" 2>&1 || exit $?
python3 "$root/tools/kstats.py" "$root/gpurun_out/$name/run_results.db" | head -6
