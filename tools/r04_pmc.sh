#!/bin/bash
# Round-4 PMC passes (tools/pmc.sh): C5 f16 (both kernels), C2 (the bench's step: the fused
# launch), C3 (the bench's step). Summaries via tools/pmc_summary.py. Usage (via gpurun):
# bash tools/r04_pmc.sh [configs...]
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
for c in ${@:-c5h c2 c3}; do
  case $c in c5h) extra="";; *) extra="--only chain";; esac
  echo "== $c $(date +%T)"
  bash tools/pmc.sh gpurun_out/pmc_$c $c $extra || exit $?
  python3 tools/pmc_summary.py gpurun_out/pmc_$c > gpurun_out/pmc_$c.txt || exit $?
done
