#!/bin/bash
# Non-temporal TX stores (tx_nt_below) on and off (MODEM_TX_NT=0) for each bench config, in-tree
# library. Usage (via gpurun): bash tools/ab_nt.sh
cd ${GRAFT_REPO_ROOT:-.}
for cfg in c5 c5h c4 c3; do
  echo "== $cfg"
  CFG=$cfg bash tools/ab_bench.sh "nt;;" "off;;MODEM_TX_NT=0" || exit $?
done
