# C2 bench lines: two launches (cur) vs the fused launch (probe variant, no probe flags)
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in cur probe cur probe; do
  RUST_MODEM_AMD_LIB=$PWD/rust-modem_amd/build/var/$v/libmodem_hip.so timeout -k 10 120 python3 bench.py --config c2 --no-cpu-baseline > gpurun_out/c2_$v.json 2> gpurun_out/c2_$v.err || exit $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/c2_$v.json')); c=d['chain_roofline']; print('$v', d['value'], d['ms_per_step'], c['tx_ms'], c['rx_ms'], c['chain_ms'], c['frac'], d['decisions_match_sent'])"
done
