# fused chain: parity tests on the in-tree library, then the kernel legs (probe variant)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_chain_fused.py -v --timeout 200 --timeout-method thread > gpurun_out/fused_tests.log 2>&1
rc=$?
tail -16 gpurun_out/fused_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
CFG=c3 REPS=50 PK="--only chain" bash tools/ab.sh "cur;;cur" "full;MODEM_CHAIN_PROBE=0;probe" "txonly;MODEM_CHAIN_PROBE=1;probe" "rxonly;MODEM_CHAIN_PROBE=2;probe" "cur2;;cur" "full2;MODEM_CHAIN_PROBE=0;probe"
