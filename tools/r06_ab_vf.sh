# Round 6: the MFMA accumulators in VGPRs (-mllvm -amdgpu-mfma-vgpr-form=1, build/var/vf) against the
# in-tree library: tests with the variant, then bench lines alternated three times.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r06o}; mkdir -p $o
V=$PWD/rust-modem_amd/build/var/vf/libmodem_hip.so
RUST_MODEM_AMD_LIB=$V timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_chain_fused.py tests/test_gpu_range.py tests/test_gpu_c5.py -x -q --timeout 300 --timeout-method thread > $o/vf_tests.txt 2>&1 || { tail -30 $o/vf_tests.txt; exit 1; }
tail -1 $o/vf_tests.txt
OUT=${OUT:-r06o}/ab VARIANTS="tree vf" CONFIGS="c3 c5h c5 c2" REPS=3 bash tools/ab_variants.sh
