#!/usr/bin/env bash
# head-dim-128 attention: numerics (attention + dropout + engine preset shapes), then the full
# attention test set and timers for the 64-wide kernels (regression check)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/hd128
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -v --timeout 200 --timeout-method thread -k "128" > $OUT/pytest_128.log 2>&1 || { tail -40 $OUT/pytest_128.log; exit 1; }
grep -cE "PASSED" $OUT/pytest_128.log
timeout -k 10 600 python -u -m pytest tests/test_attention_gpu.py tests/test_kernels_gpu.py tests/test_dropout.py tests/test_engine_gpu.py tests/test_deterministic_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu > $OUT/pytest_all.log 2>&1 || { tail -40 $OUT/pytest_all.log; exit 1; }
tail -1 $OUT/pytest_all.log
for b in 32 128; do timeout -k 10 60 bench/native/bin/fwd_new $b fwd; timeout -k 10 60 bench/native/bin/bwd_new $b bwd; done
