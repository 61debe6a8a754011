#!/usr/bin/env bash
# Tiled AdamW (8 loads in flight per thread, branch-free full-tile stores) vs the grid-stride kernel;
# GELU forward now tiled by default.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LLMT_ADAMW_TILED=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_graph_step_gpu.py \
  -x -q --timeout 120 --timeout-method thread -k "adamw or engine or gelu or graph" > gpurun_out/adamw_tests.log 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/adamw_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/adamw_tests.log)"
bash scripts/abn.sh "LLMT_ADAMW_TILED=0" "LLMT_ADAMW_TILED=1" -- --steps 20 --warmup 4 --micro-batch 32 | tee gpurun_out/ab_adamw_tiled_mb32.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/adamw_prof -o run -- python3 bench.py --steps 5 --warmup 2 --micro-batch 32 > gpurun_out/adamw_prof.log 2>&1
