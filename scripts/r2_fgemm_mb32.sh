#!/usr/bin/env bash
# Fused-GEMM A-size threshold at the presets' micro-batch 32 (default 64 MB).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/abn.sh "LLMTRAIN_FGEMM_MAX_A_MB=64" "LLMTRAIN_FGEMM_MAX_A_MB=256" "LLMTRAIN_FGEMM_MAX_A_MB=1" -- --steps 20 --warmup 4 --micro-batch 32 | tee gpurun_out/ab_fgemm_threshold_mb32.txt
