#!/bin/bash
# Round-4 evidence pass on one box (via gpurun): the chain byte-pattern floor, FETCH_SIZE width
# calibration, the new GPU tests, the flow A/B on C3 and the C3 / C5h / C2 bench lines.
# Stops at the first failing step. Usage: bash tools/r04_probe.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { echo "== $1 $(date +%T)"; }
if [ -z "$SKIP_FLOOR" ]; then
step floor;  timeout -k 10 300 tools/ubench/chain_floor > gpurun_out/floor.txt 2>&1 || exit $?
step fcal;   timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/fcal -o run -- tools/ubench/fetch_cal > gpurun_out/fcal.log 2>&1 || exit $?
fi
if [ -z "$SKIP_FLOOR" ]; then
step floorpmc; timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/floorpmc_f -o run -- tools/ubench/chain_floor pmc > gpurun_out/floorpmc_f.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/floorpmc_w -o run -- tools/ubench/chain_floor pmc > gpurun_out/floorpmc_w.log 2>&1 || exit $?
fi
step tests;  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_chain_fused.py tests/test_gpu_c5.py tests/test_gpu_range.py tests/test_gpu_nt.py tests/test_gpu_parity.py tests/test_segments.py > gpurun_out/t1.log 2>&1 || exit $?
step ab;     CFG=c3 STEPS=200 bash tools/ab_bench.sh "two;;" "flow0;;MODEM_CHAIN_FLOW=1" "flow1;;MODEM_CHAIN_FLOW=2" > gpurun_out/ab_flow.txt 2>&1 || exit $?
step c3;     timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b1.json 2>gpurun_out/b1.err || exit $?
step c5h;    timeout -k 10 200 python bench.py --config c5h --no-cpu-baseline > gpurun_out/b1c5h.json 2>gpurun_out/b1c5h.err || exit $?
step c2;     timeout -k 10 200 python bench.py --config c2 --no-cpu-baseline > gpurun_out/b1c2.json 2>gpurun_out/b1c2.err || exit $?
step done
