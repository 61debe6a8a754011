#!/usr/bin/env bash
# backward A/B: previous build vs current (timers, 2 rounds), probe, attention tests
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/bwdA
mkdir -p $OUT
BIN=bench/native/bin
for r in 1 2; do
  for v in bwd_prev bwd_new; do
    for b in 32 128; do timeout -k 10 60 $BIN/$v $b $v | tee -a $OUT/ab.log; done
  done
done
timeout -k 10 60 $BIN/bwd_new_probe 32 probe > $OUT/probe.log 2>&1
grep -E "grid|mean|kb=0" $OUT/probe.log | cut -c1-300
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_kernels_gpu.py tests/test_deterministic_gpu.py -k "attention or attn or column_sums or bitwise" -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
