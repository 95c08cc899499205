# Round 6: the GPU suite on the in-tree library (VGPR-form MFMA build), then C4's group size and TX
# store policy on the current library (rotation + TX epilogue), alternated twice.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r06p}; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.txt 2>&1 || { tail -30 $o/gpu_tests.txt; exit 1; }
tail -1 $o/gpu_tests.txt
B="--steps 100 --warmup 30 --settle-ms 200 --no-cpu-baseline --no-out-of-cache"
for rep in 1 2; do
  for v in "8:2" "4:2" "8:0" "2:2"; do
    g=${v%%:*}; nt=${v#*:}
    MODEM_TX_NT=$nt timeout -k 10 300 python3 bench.py --config c4 --group $g $B > $o/c4_g${g}_nt$nt.json 2> $o/err || { tail -3 $o/err; exit 1; }
    python3 -c "
import json;d=json.loads([l for l in open('$o/c4_g${g}_nt$nt.json') if l.startswith('{')][-1]);c=d['chain_roofline']
print('c4 group $g MODEM_TX_NT=$nt', d['value'], d['ms_per_step'], round(d['value']*18.75/8000/1000,4), 'tx', c['tx_ms'], 'rx', c['rx_ms'], 'chain', c['chain_ms'], d['decisions_match_sent'])" | tee -a $o/lines.txt
  done
done
