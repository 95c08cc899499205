# C2 fused chain probes (kernel durations under rocprofv3): where the time goes
export TMPDIR=/tmp
mkdir -p gpurun_out
CFG=c2 REPS=200 PK="--only chain" bash tools/ab.sh "full;MODEM_CHAIN_PROBE=0;probe" "notail;MODEM_CHAIN_PROBE=4;probe" "txonly;MODEM_CHAIN_PROBE=1;probe" "rxonly;MODEM_CHAIN_PROBE=2;probe" "g2;MODEM_CHAIN_GRID_DIV=2;probe" "g4;MODEM_CHAIN_GRID_DIV=4;probe" "full2;MODEM_CHAIN_PROBE=0;probe"
