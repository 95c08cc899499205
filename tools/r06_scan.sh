# Round 6: the scanned phasors' channel-parallel scan: their tests, then the rates (single channel
# vs a bank of 64) with the kernel trace.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r06f}; mkdir -p $o
timeout -k 10 300 python3 -u -m pytest tests/test_stateful.py -x -q --timeout 200 --timeout-method thread > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/scan_trace -o run -- python3 tools/scan_rate.py $SCAN_ARGS > $o/scan_rate.txt 2>&1 || { tail -20 $o/scan_rate.txt; exit 1; }
grep phasor $o/scan_rate.txt
grep -h "tx_scan\|tx_phasor" $o/scan_trace/*kernel_stats.csv | cut -c1-160
