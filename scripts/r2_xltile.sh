#!/usr/bin/env bash
# Weight-gradient tile choice: cost model (128-tile rate 0.6 PF) vs forced 128 / 256 tiles.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k wgrad \
  > gpurun_out/wgrad_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/wgrad_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/wgrad_tests.log)"
bash scripts/abn.sh "LLMT_WGRAD_TILE=0" "LLMT_WGRAD_TILE=256" -- --model gpt2-xl --micro-batch 16 --grad-accum 2 --steps 6 --warmup 2 | tee gpurun_out/ab_xl_wgrad_tile_model_vs256.txt
bash scripts/abn.sh "LLMT_WGRAD_TILE=0" "LLMT_WGRAD_TILE=256" -- --micro-batch 32 --steps 20 --warmup 4 | tee gpurun_out/ab_mb32_wgrad_tile_model_vs256.txt
