#!/bin/bash
# persistent, software-pipelined cross-entropy (LLMT_CE_PERSIST=1): numerics, op time, step A/B
set -eo pipefail
O=gpurun_out/s28
mkdir -p $O
LLMT_CE_PERSIST=1 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k cross_entropy > $O/pytest_ce.txt 2>&1
for r in 1 2; do
  for p in 0 1; do
    LLMT_CE_PERSIST=$p timeout -k 10 120 python -u bench/ce_one.py 2>&1 | grep '^{' | sed "s/^/persist$p /" >> $O/ce_one.txt
  done
done
bash scripts/abn.sh "LLMT_CE_PERSIST=0" "LLMT_CE_PERSIST=1" -- --steps 10 --warmup 3 > $O/ab_mb128.txt 2>&1
bash scripts/abn.sh "LLMT_CE_PERSIST=0" "LLMT_CE_PERSIST=1" -- --micro-batch 32 --steps 20 --warmup 5 > $O/ab_mb32.txt 2>&1
