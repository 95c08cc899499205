# Round 6: the cleaned-up sources (experiment switches removed, variants in their own units, the RX
# window descriptor bounded by the call's buffer): GPU suite with the new window-bounds test, then
# the C4 batch-vs-single probe and C3 lines.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/r06c; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.txt 2>&1 || { tail -30 $o/gpu_tests.txt; exit 1; }
tail -1 $o/gpu_tests.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.txt 2>&1 || { tail -20 $o/smoke.txt; exit 1; }
tail -1 $o/smoke.txt
bash tools/r06_probe_c4b.sh || exit 1
OUT=r06c/ab VARIANTS=tree CONFIGS="c3 c4 c5 c5h c2" REPS=1 DRV=3 bash tools/ab_variants.sh
