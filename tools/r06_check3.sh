# Round 6: the GPU suite and smoke on the in-tree library (TX epilogue: no unscale selects, exact f32
# index split, bits prefetch through a descriptor), C5 f16 TX traffic, every config's line and three
# driver-style C3 lines.
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r06n}; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.txt 2>&1 || { tail -30 $o/gpu_tests.txt; exit 1; }
tail -1 $o/gpu_tests.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.txt 2>&1 || { tail -20 $o/smoke.txt; exit 1; }
tail -1 $o/smoke.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/pmc_c5h/p1 -o run -- python3 tools/prof_kernels.py --config c5h --reps 4 --only tx > $o/pmc_c5h.log 2>&1 || { tail -5 $o/pmc_c5h.log; exit 1; }
python3 tools/pmc_summary.py $o/pmc_c5h | grep -A1 tx_mfma
OUT=${OUT:-r06n}/ab VARIANTS="tree" CONFIGS="c3 c4 c5 c5h c2" REPS=1 DRV=3 bash tools/ab_variants.sh
