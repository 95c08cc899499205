# The GPU test suite on one box (round-end style), output under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gputests.log 2>&1
rc=$?
tail -5 gpurun_out/gputests.log
exit $rc
