# Round 6: the batch launches' per-channel workgroup rotation (MODEM_BATCH_ROT) against none, C4
# batch probes and the C4 job, alternated twice.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r06d}; mkdir -p $o
for rep in 1 2; do
  for rot in 0 1; do
    for w in "qpsk 2 65 4 4194304 4 --label batch4x22_rot$rot" "qpsk 2 65 4 2097152 8 --label batch8x21_rot$rot"; do
      MODEM_BATCH_ROT=$rot timeout -k 10 120 python3 tools/wl_probe.py $w >> $o/probe.txt 2>> $o/err || { tail -5 $o/err; exit 1; }
      tail -1 $o/probe.txt
    done
  done
done
OUT=${OUT:-r06d}/ab VARIANTS="tree:MODEM_BATCH_ROT=0 tree" CONFIGS="c4" REPS=2 bash tools/ab_variants.sh
