# Round 6: WRITE_SIZE calibration by store width and pattern (tools/ubench/write_cal.hip).
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r06l}; mkdir -p $o
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/wcal -o run -- tools/ubench/write_cal > $o/wcal.log 2>&1 || { tail -5 $o/wcal.log; exit 1; }
python3 tools/pmc_summary.py $o/wcal
