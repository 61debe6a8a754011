#!/usr/bin/env bash
# fused delta in the attention backward: timers (delta kernel vs fused, 2 rounds) + GPU tests
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/fdelta
mkdir -p $OUT
for r in 1 2; do
  for f in 0 1; do
    for b in 32 128; do LLMT_ATTN_FUSED_DELTA=$f timeout -k 10 60 bench/native/bin/bwd_new $b "fused_delta=$f" | tee -a $OUT/ab.log; done
  done
done
timeout -k 10 600 python -u -m pytest tests/test_attention_gpu.py tests/test_kernels_gpu.py tests/test_dropout.py tests/test_engine_gpu.py tests/test_deterministic_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
