#!/bin/bash
# Round 5: validate the chain-batch lanes test and the 500 ms settle on one box.
set -o pipefail
O=gpurun_out/r05v1; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_chain_batch.py > $O/tests.txt 2>&1 &&
for i in 1 2 3; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/drv$i.json 2> $O/drv$i.err || exit 1; done &&
timeout -k 10 200 python bench.py --config c4 --steps 20 --warmup 5 > $O/c4.json 2> $O/c4.err
