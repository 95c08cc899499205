# A/B of RX variants (tools/build_var.sh builds) on one box: dispatch ubench, rocprof kernel
# stats, stamps, driver-style bench lines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/rust-modem_amd/build/var
timeout -k 10 60 tools/ubench/bin/dispatch > gpurun_out/dispatch.txt 2>&1 && echo dispatch-ok || exit 1
for v in ${VARS:-base dyn base dyn}; do
  RUST_MODEM_AMD_LIB=$V/$v/libmodem_hip.so timeout -k 10 120 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-out-of-cache > gpurun_out/pb_$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/pb_$v.json'));c=d['chain_roofline'];print('$v', d['value'], d['ms_per_step'], 'tx',c['tx_ms'],'rx',c['rx_ms'],'chain',c['chain_ms'],'rxin',c['rx_in_chain_ms'],d['decisions_match_sent'])"
done
CFG=c3 REPS=50 bash tools/ab.sh ${AB:-"base;;base" "dyn;;dyn" "base2;;base" "dyn2;;dyn"} || exit 1
RUST_MODEM_AMD_LIB=$V/${SV:-dynstamps}/libmodem_hip.so timeout -k 10 150 python3 -u tools/stamps.py --tag ${SV:-dynstamps} > gpurun_out/stamps_${SV:-dynstamps}.txt 2>&1 && echo stamps-ok
