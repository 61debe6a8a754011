#!/usr/bin/env bash
# Side-stream weight gradients on the 128x128-tile kernel (104 VGPRs, 64 KB LDS) vs the cost model.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/abn.sh "LLMTRAIN_WGRAD_SIDE_TILE=0" "LLMTRAIN_WGRAD_SIDE_TILE=128" -- --steps 15 --warmup 4 | tee gpurun_out/ab_side_tile_mb128.txt
bash scripts/abn.sh "LLMTRAIN_WGRAD_SIDE_TILE=0" "LLMTRAIN_WGRAD_SIDE_TILE=128" -- --steps 20 --warmup 4 --micro-batch 32 | tee gpurun_out/ab_side_tile_mb32.txt
