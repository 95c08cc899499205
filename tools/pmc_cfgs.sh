#!/bin/bash
# PMC passes (tools/pmc.sh) for the out-of-cache configs; traffic per launch into gpurun_out.
# Usage (via gpurun): bash tools/pmc_cfgs.sh <tag>
set -o pipefail
tag=${1:-pmccfg}; cd ${GRAFT_REPO_ROOT:-.}
for c in c5 c4; do
  bash tools/pmc.sh gpurun_out/$tag/$c $c || exit $?
  python3 tools/pmc_summary.py gpurun_out/$tag/$c > gpurun_out/$tag/${c}_summary.txt || exit 1
done
