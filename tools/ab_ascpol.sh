#!/bin/bash
# RX tile order by size (rx_asc_rounds) on and off (MODEM_RX_ASC=0) per bench config, in-tree
# library; then the GPU tests that cover large RX calls. Usage (via gpurun).
cd ${GRAFT_REPO_ROOT:-.}
for cfg in c5 c4 c5h; do
  echo "== $cfg"
  CFG=$cfg bash tools/ab_bench.sh "asc;;" "off;;MODEM_RX_ASC=0" || exit $?
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_nt.py tests/test_gpu_c4.py tests/test_gpu_range.py -x -q --timeout 250 --timeout-method thread > gpurun_out/asc_tests.log 2>&1; rc=$?; tail -2 gpurun_out/asc_tests.log; exit $rc
