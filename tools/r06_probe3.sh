# Round 6: straddling buffer stores, and C5 f16 RX WRITE_SIZE without its I/Q stores / without its
# decision stores (timing-probe builds), against the in-tree library.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r06j}; mkdir -p $o
timeout -k 5 60 tools/ubench/oob_store > $o/oob_store.txt 2>&1 || { cat $o/oob_store.txt; exit 1; }
cat $o/oob_store.txt
for v in tree noiq nosym; do
  lib=""; [ $v != tree ] && lib=$PWD/rust-modem_amd/build/var/$v/libmodem_hip.so
  RUST_MODEM_AMD_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/pmc_$v/p1 -o run -- python3 tools/prof_kernels.py --config c5h --reps 4 --only rx > $o/pmc_$v.log 2>&1 || { tail -5 $o/pmc_$v.log; exit 1; }
  echo "== $v"; python3 tools/pmc_summary.py $o/pmc_$v | grep -A1 "rx_mfma"
done
