#!/bin/bash
# A/B by the bench's own legs (TX alone, RX alone re-reading its resident input, the chain):
# bench.py per case "label;variant;ENV=val ..." (variant: a tools/build_var.sh build, empty =
# in-tree library), config CFG (default c5), alternated twice. Usage (via gpurun): bash tools/ab_bench.sh cases...
cd ${GRAFT_REPO_ROOT:-.}
cfg=${CFG:-c5}
mkdir -p gpurun_out/abb
for rep in 1 2; do
  for c in "$@"; do
    IFS=';' read -r label var envs <<< "$c"
    lib=""; [ -n "$var" ] && lib="$PWD/rust-modem_amd/build/var/$var/libmodem_hip.so"
    env $envs RUST_MODEM_AMD_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --steps ${STEPS:-100} --warmup 20 --settle-ms 0 \
        --no-cpu-baseline --no-out-of-cache > gpurun_out/abb/$label.$rep.json 2> gpurun_out/abb/$label.$rep.err
    rc=$?
    case $rc in 0) ;; *) echo "$label rc=$rc"; tail -5 gpurun_out/abb/$label.$rep.err; exit $rc;; esac
    python3 -c "import json;d=json.load(open('gpurun_out/abb/$label.$rep.json'));c=d['chain_roofline'];print('$label', d['value'], 'tx',c['tx_ms'],'rx',c['rx_ms'],'chain',c['chain_ms'],'rx_in_chain',c['rx_in_chain_ms'], 'ok', d['decisions_match_sent'])"
  done
done
