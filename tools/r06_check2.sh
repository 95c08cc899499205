# Round 6: the GPU suite (window bounds, scan batch), the scan rates (+ their kernel trace), and the
# batch workgroup rotation A/B (tools/r06_rot.sh).
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r06e}; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.txt 2>&1 || { tail -30 $o/gpu_tests.txt; exit 1; }
tail -1 $o/gpu_tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/scan_trace -o run -- python3 tools/scan_rate.py > $o/scan_rate.txt 2>&1 || { tail -20 $o/scan_rate.txt; exit 1; }
grep phasor $o/scan_rate.txt
grep -h "tx_scan\|tx_phasor" $o/scan_trace/*kernel_stats.csv | cut -c1-200
OUT=${OUT:-r06e}/rot bash tools/r06_rot.sh
