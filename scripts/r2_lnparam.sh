#!/usr/bin/env bash
# Timing experiment: LayerNorm backward without the gamma/beta column partials (LLMT_LN_BWD_LEAN=3,
# 80 VGPRs: two waves fit beside the side stream's weight-gradient GEMM) vs the lean kernel.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 3; do echo "solo lean=$v: $(LLMT_LN_BWD_LEAN=$v timeout -k 10 120 python bench/micro.py ln 131072 | grep ln_bwd)"; done
bash scripts/abn.sh "LLMT_LN_BWD_LEAN=1" "LLMT_LN_BWD_LEAN=3" -- --steps 15 --warmup 4 | tee gpurun_out/ab_ln_noparam_mb128.txt
bash scripts/abn.sh "LLMT_LN_BWD_LEAN=1" "LLMT_LN_BWD_LEAN=3" -- --steps 20 --warmup 4 --micro-batch 32 | tee gpurun_out/ab_ln_noparam_mb32.txt
