# Round 6: the TX epilogue without the conditional unscale's selects, with the exact f32 index split
# and the bits prefetch through a buffer descriptor (build/var/txv, MODEM_VARIANTS_MIN): TX parity
# tests with the variant, then the bench A/B against the in-tree library.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r06m}; mkdir -p $o
V=$PWD/rust-modem_amd/build/var/txv/libmodem_hip.so
RUST_MODEM_AMD_LIB=$V timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_chain_fused.py tests/test_gpu_range.py tests/test_gpu_nt.py tests/test_gpu_chain_batch.py tests/test_segments.py -x -q --timeout 300 --timeout-method thread > $o/txv_tests.txt 2>&1 || { tail -30 $o/txv_tests.txt; exit 1; }
tail -1 $o/txv_tests.txt
OUT=${OUT:-r06m}/ab VARIANTS="tree txv" CONFIGS="c3 c5h c5 c2" REPS=3 DRV=0 bash tools/ab_variants.sh
