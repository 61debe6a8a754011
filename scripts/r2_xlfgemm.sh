#!/usr/bin/env bash
# GPT-2 XL: hand-written fused forward/dX GEMMs (default) vs hipBLASLt + separate GELU passes.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/abn.sh "LLMTRAIN_FUSED_GEMM=1" "LLMTRAIN_FUSED_GEMM=0" "LLMTRAIN_FUSED_GEMM=fwd" -- --model gpt2-xl --micro-batch 16 --grad-accum 2 --steps 6 --warmup 2 | tee gpurun_out/ab_xl_fused_gemm.txt
