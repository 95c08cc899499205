#!/bin/bash
# Round 5: PMC passes of C5 f16 and C5 f32 with the wide TX tiles (LDS bank conflicts, VALU and
# MFMA activity of both kernels), one counter group per rocprofv3 run.
cd ${GRAFT_REPO_ROOT:-.}
tools/pmc.sh gpurun_out/r05h/pmc_c5h c5h && tools/pmc.sh gpurun_out/r05h/pmc_c5 c5 &&
python3 tools/pmc_summary.py gpurun_out/r05h/pmc_c5h > gpurun_out/r05h/c5h_summary.txt &&
python3 tools/pmc_summary.py gpurun_out/r05h/pmc_c5 > gpurun_out/r05h/c5_summary.txt &&
timeout -k 10 120 tools/ubench/valu_rates > gpurun_out/r05h/valu_rates.txt 2>&1
