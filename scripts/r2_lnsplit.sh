#!/usr/bin/env bash
# Split-row LayerNorm backward for wide rows (GPT-2 XL): numerics, then same-box A/B.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LLMT_LN_BWD_SPLIT=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q \
  --timeout 120 --timeout-method thread -k "layernorm or engine" > gpurun_out/lnsplit_tests.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/lnsplit_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/lnsplit_tests.log)"
bash scripts/abn.sh "LLMT_LN_BWD_SPLIT=0" "LLMT_LN_BWD_SPLIT=1" -- --model gpt2-xl --micro-batch 16 --grad-accum 2 --steps 6 --warmup 2 | tee gpurun_out/ab_ln_split_xl.txt
