#!/usr/bin/env bash
# Lean LayerNorm backward: numerics under each variant, solo timing, in-step A/B.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 1 2; do
  LLMT_LN_BWD_LEAN=$v timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q \
    --timeout 120 --timeout-method thread -k "layernorm or ln or engine or resume" > gpurun_out/ln_tests_$v.log 2>&1 \
    || { echo "tests failed (lean=$v)"; tail -30 gpurun_out/ln_tests_$v.log; exit 1; }
  echo "lean=$v: $(tail -1 gpurun_out/ln_tests_$v.log)"
done
for v in 0 1 2; do
  echo "solo lean=$v M=131072: $(LLMT_LN_BWD_LEAN=$v timeout -k 10 120 python bench/micro.py ln 131072 | grep ln_bwd)"
  echo "solo lean=$v M=32768: $(LLMT_LN_BWD_LEAN=$v timeout -k 10 120 python bench/micro.py ln 32768 | grep ln_bwd)"
done
bash scripts/abn.sh "LLMT_LN_BWD_LEAN=0" "LLMT_LN_BWD_LEAN=1" "LLMT_LN_BWD_LEAN=2" -- --steps 15 --warmup 4 | tee gpurun_out/ab_ln_lean_mb128.txt
bash scripts/abn.sh "LLMT_LN_BWD_LEAN=0" "LLMT_LN_BWD_LEAN=1" "LLMT_LN_BWD_LEAN=2" -- --steps 20 --warmup 4 --micro-batch 32 | tee gpurun_out/ab_ln_lean_mb32.txt
