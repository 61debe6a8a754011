#!/usr/bin/env bash
# Cross-entropy / GELU forward with every row load in flight: numerics, solo timing, in-step A/B.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for o in 6 5; do
  LLMT_CE_OCC=$o timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q \
    --timeout 120 --timeout-method thread -k "cross_entropy or gelu or engine" > gpurun_out/ce_tests_$o.log 2>&1 \
    || { echo "tests failed"; tail -30 gpurun_out/ce_tests_$o.log; exit 1; }
  echo "occ=$o tests: $(tail -1 gpurun_out/ce_tests_$o.log)"
  echo "occ=$o solo: $(LLMT_CE_OCC=$o timeout -k 10 120 python bench/ce_one.py 131072 | tail -1)"
done
echo "gelu solo: $(timeout -k 10 120 python bench/micro.py ln 131072 | grep gelu | tr '\n' ' ')"
bash scripts/abn.sh "LLMT_CE_OCC=6" "LLMT_CE_OCC=5" -- --steps 15 --warmup 4 | tee gpurun_out/ab_ce_occ_mb128.txt
