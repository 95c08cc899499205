# Round 6: the partial out-of-range buffer store probe, then C5 f16's traffic (FETCH_SIZE and
# WRITE_SIZE passes, one rocprofv3 run each) on the current library.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r06h}; mkdir -p $o
timeout -k 5 60 tools/ubench/oob_store > $o/oob_store.txt 2>&1 || { cat $o/oob_store.txt; exit 1; }
cat $o/oob_store.txt
i=0
for ctr in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $o/pmc_c5h/p$i -o run -- python3 tools/prof_kernels.py --config c5h --reps 4 > $o/pmc_c5h.$ctr.log 2>&1 || { tail -5 $o/pmc_c5h.$ctr.log; exit 1; }
done
python3 tools/pmc_summary.py $o/pmc_c5h > $o/pmc_c5h.txt && cat $o/pmc_c5h.txt
