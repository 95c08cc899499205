# fused chain probes: why the fused kernel's TX part is slower; C2 fused vs two launches
export TMPDIR=/tmp
mkdir -p gpurun_out
MODEM_CHAIN_VERBOSE=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_chain_fused.py -x -v --timeout 200 --timeout-method thread > gpurun_out/fused_tests.log 2>&1
rc=$?
tail -16 gpurun_out/fused_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
CFG=c3 REPS=50 PK="--only chain" bash tools/ab.sh "cur;;cur" "tx1;MODEM_CHAIN_PROBE=1;probe" "tx5;MODEM_CHAIN_PROBE=5;probe" "tx13;MODEM_CHAIN_PROBE=13;probe" "full;MODEM_CHAIN_PROBE=0;probe" || exit $?
CFG=c2 REPS=200 PK="--only chain" bash tools/ab.sh "c2cur;;cur" "c2full;MODEM_CHAIN_PROBE=0;probe" "c2cur2;;cur" "c2full2;MODEM_CHAIN_PROBE=0;probe"
