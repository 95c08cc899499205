# Round 6: C4's batch launches against one channel: where does the batch's per-sample cost come from?
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r06b}; mkdir -p $o
for w in "qpsk 2 65 4 16777216 1 --label single24" "qpsk 2 65 4 16777216 1 --batch --label batch1x24" \
         "qpsk 2 65 4 4194304 1 --label single22" "qpsk 2 65 4 8388608 2 --label batch2x23" \
         "qpsk 2 65 4 4194304 4 --label batch4x22" "qpsk 2 65 4 2097152 8 --label batch8x21" \
         "qam16 4 129 4 16777216 1 --batch --label c3batch1" "qam16 4 129 4 16777216 1 --label c3single"; do
  timeout -k 10 120 python3 tools/wl_probe.py $w >> $o/probe.txt 2>> $o/err || { tail -5 $o/err; exit 1; }
  tail -1 $o/probe.txt
done
