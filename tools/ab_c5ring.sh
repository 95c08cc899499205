#!/bin/bash
# A/B: C5 RX, RxMfma (base build) against the block-ring kernel (ring build); kernel-trace stats
# of tools/prof_kernels.py with its poisoned-output loopback check. Usage (via gpurun).
cd ${GRAFT_REPO_ROOT:-.}
CFG=c5 REPS=10 bash tools/ab.sh "ring;;ring" "base;;base" "ring2;;ring" "base2;;base"
