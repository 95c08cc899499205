# A/B on one box: base vs fix2 with static tile order (MODEM_RX_STATIC=1) vs fix2 dynamic pools.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/rust-modem_amd/build/var
line() {   # label env lib
  env $2 RUST_MODEM_AMD_LIB=$V/$3/libmodem_hip.so timeout -k 10 120 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-out-of-cache > gpurun_out/pb_$1.json 2>/dev/null || return 1
  python3 -c "import json;d=json.load(open('gpurun_out/pb_$1.json'));c=d['chain_roofline'];print('$1', d['value'], d['ms_per_step'], 'tx',c['tx_ms'],'rx',c['rx_ms'],'chain',c['chain_ms'],'rxin',c['rx_in_chain_ms'],d['decisions_match_sent'])"
}
for r in 1 2; do
  line base$r X=1 base || exit 1
  line stat$r MODEM_RX_STATIC=1 fix2 || exit 1
  line dyn$r X=1 fix2 || exit 1
done
for c in c2 c3; do
  CFG=$c REPS=50 bash tools/ab.sh "${c}_base;;base" "${c}_stat;MODEM_RX_STATIC=1;fix2" "${c}_dyn;;fix2" || exit 1
done
RUST_MODEM_AMD_LIB=$V/fix2stamps/libmodem_hip.so timeout -k 10 150 python3 -u tools/stamps.py --tag fix2dyn > gpurun_out/stamps_fix2dyn.txt 2>&1 && echo stamps-dyn-ok || exit 1
MODEM_RX_STATIC=1 RUST_MODEM_AMD_LIB=$V/fix2stamps/libmodem_hip.so timeout -k 10 150 python3 -u tools/stamps.py --tag fix2stat > gpurun_out/stamps_fix2stat.txt 2>&1 && echo stamps-stat-ok
