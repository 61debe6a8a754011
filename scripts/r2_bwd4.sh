#!/usr/bin/env bash
# 4-wave vs 8-wave attention backward: timers (both kernels, B=32/128), then the GPU attention tests
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/bwd4
mkdir -p $OUT
BIN=bench/native/bin
for r in 1 2; do
  for w in 8 4; do
    for b in 32 128; do LLMT_ATTN_BWD_WAVES=$w timeout -k 10 60 $BIN/bwd_new $b "waves$w" | tee -a $OUT/ab.log; done
  done
done
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_kernels_gpu.py -k "attention or attn" -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
