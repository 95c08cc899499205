export TMPDIR=/tmp
mkdir -p gpurun_out
RUST_MODEM_AMD_LIB=$PWD/rust-modem_amd/build/var/fused/libmodem_hip.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_chain_fused.py -v --timeout 120 --timeout-method thread > gpurun_out/fused_tests.log 2>&1
rc=$?
tail -20 gpurun_out/fused_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
CFG=c3 REPS=50 PK="--only chain" bash tools/ab.sh "c1;;cur" "f1;;fused" "c2;;cur" "f2;;fused"
