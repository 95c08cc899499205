set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 90 tools/ubench/bin/valu_rates > gpurun_out/valu_rates.txt 2>&1 && echo ubench-ok &&
RUST_MODEM_AMD_LIB=$PWD/rust-modem_amd/build/var/stamps/libmodem_hip.so timeout -k 10 150 python3 -u tools/stamps.py --tag base > gpurun_out/stamps_base.txt 2>&1 && echo stamps-ok &&
timeout -k 10 180 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r03_a.json 2> gpurun_out/bench_r03_a.err && echo bench-ok &&
timeout -k 10 180 python3 -u bench.py --gpus 2 --config c4 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r03_g2.json 2> gpurun_out/bench_r03_g2.err && echo g2-ok
