#!/bin/bash
# Round-5 probe (via gpurun): the chains' byte-pattern floors (tools/ubench/chain_floor), the
# fused-chain tests after the hand-off window swizzle, bench lines for C2, C4 (the 64-channel
# job in groups of 8 and of 4) and C3 (driver-style), C2's LDS bank conflicts and C4's traffic.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/r05a; mkdir -p $o
set -o pipefail
step() { local name=$1; shift; echo "== $name $(date +%T)"; "$@"; local rc=$?; echo "   rc=$rc"; return $rc; }
step floor timeout -k 10 300 tools/ubench/chain_floor all > $o/floor.txt 2>&1 || exit $?
step fused timeout -k 10 300 python3 -u -m pytest tests/test_gpu_chain_fused.py -x -q --timeout 120 --timeout-method thread > $o/fused_tests.log 2>&1 || exit $?
B="--steps 200 --warmup 50 --no-cpu-baseline --no-out-of-cache"
step c2 timeout -k 10 300 python3 bench.py --config c2 $B > $o/c2.json 2> $o/c2.err || exit $?
for g in 8 4; do
  step c4g$g timeout -k 10 300 python3 bench.py --config c4 --group $g $B > $o/c4_g$g.json 2> $o/c4_g$g.err || exit $?
done
step c3drv timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-out-of-cache > $o/c3_drv.json 2> $o/c3_drv.err || exit $?
step pmc_c2 timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS_LDS --output-format csv -d $o/pmc_c2 -o run -- python3 tools/prof_kernels.py --config c2 --only chain --reps 10 > $o/pmc_c2.log 2>&1 || exit $?
step pmc_c4_fetch timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/pmc_c4f -o run -- python3 tools/prof_kernels.py --config c4 --group 8 --reps 3 > $o/pmc_c4f.log 2>&1 || exit $?
step pmc_c4_write timeout -k 10 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/pmc_c4w -o run -- python3 tools/prof_kernels.py --config c4 --group 8 --reps 3 > $o/pmc_c4w.log 2>&1 || exit $?
echo done
