#!/usr/bin/env bash
# Fused-GEMM A/B: the shipped .so vs llmtrain/ops/_prev_hip.so (built from the previous source),
# micro timings at M = 131072 for the dX shapes; GPU tests for the fused GEMM first.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/fgab; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fused or gemm" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cp llmtrain/ops/_llmtrain_hip.so $OUT/new.so
for r in 1 2; do
  for v in prev new; do
    if [ $v = prev ]; then cp llmtrain/ops/_prev_hip.so llmtrain/ops/_llmtrain_hip.so; else cp $OUT/new.so llmtrain/ops/_llmtrain_hip.so; fi
    for sh in "768 3072 2 1" "2304 768 0 1" "768 768 0 1" "3072 768 0 1"; do
      echo -n "$v $sh "; timeout -k 10 60 python bench/micro.py fgemm1 $sh 131072 2>/dev/null
    done
  done
done
cp $OUT/new.so llmtrain/ops/_llmtrain_hip.so
