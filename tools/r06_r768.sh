# Round 6: the RX at 5 waves per SIMD — 768-instant tiles (3 filter waves of 4;
# 28 KB of LDS: 5 workgroups per CU; 95 VGPRs, no scratch) in a probe build (build/var/r768, with
# MODEM_PROBE_RX768=1 in the environment) against the default 1024-instant tiles at 4 waves per SIMD:
# C3-sized RX tests with the probe, then bench lines alternated three times.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r06q}; mkdir -p $o
V=$PWD/rust-modem_amd/build/var/r768/libmodem_hip.so
MODEM_PROBE_RX768=1 RUST_MODEM_AMD_LIB=$V timeout -k 10 600 python3 -u -m pytest tests/test_gpu_window_bounds.py "tests/test_gpu_range.py::test_c3_full_size_against_oracle" tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $o/r768_tests.txt 2>&1 || { tail -30 $o/r768_tests.txt; exit 1; }
tail -1 $o/r768_tests.txt
OUT=${OUT:-r06q}/ab VARIANTS="r768 r768:MODEM_PROBE_RX768=1" CONFIGS="c3" REPS=3 bash tools/ab_variants.sh
