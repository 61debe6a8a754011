#!/usr/bin/env bash
# attention forward iteration: kernel numerics tests, then the micro-benchmark at B=32 and B=128
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2af
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_kernels_gpu.py -k "attention" -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python bench/micro.py attn 32 > $OUT/micro_b32.log 2>&1
timeout -k 10 120 python bench/micro.py attn 128 > $OUT/micro_b128.log 2>&1
grep llmtrain $OUT/micro_b32.log $OUT/micro_b128.log
