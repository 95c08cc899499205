# C2 with the LDS hand-off fused form: chain parity tests, then the C2 bench line (x2)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_chain_fused.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread > gpurun_out/c2ho_tests.log 2>&1
rc=$?
tail -4 gpurun_out/c2ho_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/c2ho_tests.log | head -20; exit $rc; }
for k in 1 2; do
  timeout -k 10 120 python3 bench.py --config c2 --no-cpu-baseline > gpurun_out/c2ho_$k.json 2> gpurun_out/c2ho_$k.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/c2ho_$k.json')); c=d['chain_roofline']; print('c2', d['value'], d['ms_per_step'], c['tx_ms'], c['rx_ms'], c['chain_ms'], c['frac'], c['fused'], d['decisions_match_sent'])"
done
