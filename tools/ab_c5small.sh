cd $GRAFT_REPO_ROOT
CFG=c5 REPS=10 bash tools/ab.sh "base;;base" "small;;small" "base2;;base" "small2;;small"
