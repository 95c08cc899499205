# Round 6: the RX's f16 I/Q pair stores (build/var/pair, MODEM_VARIANTS_MIN): tests with the variant,
# C5 f16 WRITE_SIZE of the variant, then the bench A/B against the in-tree library.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r06i}; mkdir -p $o
V=$PWD/rust-modem_amd/build/var/pair/libmodem_hip.so
RUST_MODEM_AMD_LIB=$V timeout -k 10 600 python3 -u -m pytest tests/test_gpu_range.py tests/test_gpu_nt.py tests/test_gpu_chain_fused.py tests/test_gpu_c5.py tests/test_gpu_window_bounds.py -x -q --timeout 300 --timeout-method thread > $o/pair_tests.txt 2>&1 || { tail -30 $o/pair_tests.txt; exit 1; }
tail -1 $o/pair_tests.txt
RUST_MODEM_AMD_LIB=$V timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/pmc_w/p1 -o run -- python3 tools/prof_kernels.py --config c5h --reps 4 > $o/pmc_w.log 2>&1 || { tail -5 $o/pmc_w.log; exit 1; }
python3 tools/pmc_summary.py $o/pmc_w | grep -A1 "rx_mfma\|tx_mfma"
OUT=${OUT:-r06i}/ab VARIANTS="tree pair" CONFIGS="c5h c3" REPS=3 bash tools/ab_variants.sh
