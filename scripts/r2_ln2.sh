#!/usr/bin/env bash
# add+LayerNorm forward with all loads up front, lean backward at every width: numerics, solo, A/B.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q \
  --timeout 120 --timeout-method thread -k "layernorm or ln or engine or resume" > gpurun_out/ln2_tests.log 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/ln2_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/ln2_tests.log)"
LLMT_LN_BWD_LEAN_WIDE=0 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q \
  --timeout 120 --timeout-method thread -k "layernorm" > gpurun_out/ln2_tests_wide0.log 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/ln2_tests_wide0.log; exit 1; }
for M in 131072 32768; do echo "solo M=$M: $(timeout -k 10 120 python bench/micro.py ln $M | grep ln | tr '\n' ' ')"; done
bash scripts/abn.sh "LLMT_LN_BWD_LEAN_WIDE=0" "LLMT_LN_BWD_LEAN_WIDE=1" -- --model gpt2-xl --micro-batch 16 --grad-accum 2 --steps 6 --warmup 2 | tee gpurun_out/ab_ln_lean_xl.txt
bash scripts/abn.sh "X=0" -- --steps 15 --warmup 4 | tee gpurun_out/ab_ln_fwd_mb128.txt
