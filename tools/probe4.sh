# Sensitivity A/B (extra s_nop / VALU per RX tile), C2 slow-tile fix, TX + RX stamps, new-path bench lines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/rust-modem_amd/build/var
for r in 1 2; do
  timeout -k 10 120 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-out-of-cache > gpurun_out/pb_intree$r.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/pb_intree$r.json'));c=d['chain_roofline'];print('intree$r', d['value'], d['ms_per_step'], 'tx',c['tx_ms'],'rx',c['rx_ms'],'chain',c['chain_ms'],'rxin',c['rx_in_chain_ms'],d['decisions_match_sent'], d['roofline']['frac'])"
done
CFG=c3 REPS=50 bash tools/ab.sh "c3cur;;cur" "c3snop100;;snop100" "c3valu64;;valu64" "c3cur2;;cur" "c3base;;base" || exit 1
CFG=c2 REPS=50 bash tools/ab.sh "c2base;;base" "c2cur;;cur" "c2base2;;base" "c2cur2;;cur" || exit 1
for k in rx tx; do
  RUST_MODEM_AMD_LIB=$V/curstamps/libmodem_hip.so timeout -k 10 150 python3 -u tools/stamps.py --tag cur --kernel $k > gpurun_out/stamps_cur_$k.txt 2>&1 && echo stamps-$k-ok || exit 1
done
