#!/usr/bin/env bash
# Tiled GELU forward (4 vectors per thread, loads before the first wait) vs the grid-stride kernel.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LLMT_GELU_TILED=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q \
  --timeout 120 --timeout-method thread -k "gelu or engine" > gpurun_out/gelu_tests.log 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/gelu_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/gelu_tests.log)"
for r in 1 2; do for v in 0 1; do
  echo "solo tiled=$v: $(LLMT_GELU_TILED=$v timeout -k 10 120 python bench/micro.py ln 131072 | grep gelu_fwd)"
done; done
bash scripts/abn.sh "LLMT_GELU_TILED=0" "LLMT_GELU_TILED=1" -- --steps 15 --warmup 4 | tee gpurun_out/ab_gelu_tiled_mb128.txt
