cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
mkdir -p gpurun_out/r06g
RUST_MODEM_AMD_LIB=$PWD/rust-modem_amd/build/var/sf/libmodem_hip.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_window_bounds.py tests/test_gpu_parity.py tests/test_gpu_range.py tests/test_gpu_c5.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06g/sf_tests.txt 2>&1 || { tail -30 gpurun_out/r06g/sf_tests.txt; exit 1; }
tail -1 gpurun_out/r06g/sf_tests.txt
OUT=r06g/ab VARIANTS="tree sf" CONFIGS="c3 c4 c5 c5h" REPS=3 bash tools/ab_variants.sh
