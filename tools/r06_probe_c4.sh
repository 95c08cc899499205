cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/r06a; mkdir -p $o
timeout -k 10 120 python3 tools/wl_probe.py qpsk 2 65 4 16777216 1 --label single24 >> $o/probe.txt 2>> $o/err || { tail -5 $o/err; exit 1; }
for args in "--group 4 --separate" "--group 4 --stagger 0" "--group 4 --stagger 4096" "--group 4 --stagger 266240" "--group 8 --separate" "--group 8 --stagger 0" "--group 8 --stagger 4096"; do
  timeout -k 10 150 python3 tools/c4_layout_probe.py $args >> $o/probe.txt 2>> $o/err || { tail -5 $o/err; exit 1; }
  tail -1 $o/probe.txt
done
