#!/bin/bash
# LayerNorm backward with two rows per wave (LLMT_LN_BWD_ROWS=2) now that no side stream shares the CUs
set -eo pipefail
O=gpurun_out/s30
mkdir -p $O
LLMT_LN_BWD_ROWS=2 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k layernorm > $O/pytest_ln.txt 2>&1
bash scripts/abn.sh "LLMT_LN_BWD_ROWS=1" "LLMT_LN_BWD_ROWS=2" -- --steps 10 --warmup 3 > $O/ab_mb128.txt 2>&1
bash scripts/abn.sh "LLMT_LN_BWD_ROWS=1" "LLMT_LN_BWD_ROWS=2" -- --micro-batch 32 --steps 20 --warmup 5 > $O/ab_mb32.txt 2>&1
