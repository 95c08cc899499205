cd ${GRAFT_REPO_ROOT:-.}
echo "== c3"; CFG=c3 STEPS=400 bash tools/ab_bench.sh "base;base" "rxnt;rxnt" || exit 1
echo "== c5"; CFG=c5 bash tools/ab_bench.sh "tree;;" "rxnt;rxnt" || exit 1
echo "== c4"; CFG=c4 bash tools/ab_bench.sh "tree;;" "rxnt;rxnt" || exit 1
