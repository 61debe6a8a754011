#!/usr/bin/env bash
# Lean LayerNorm backward grid: 1 / 2 / 3 (default) resident waves of workgroups.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/abn.sh "LLMT_LN_BWD_WAVES=3" "LLMT_LN_BWD_WAVES=2" "LLMT_LN_BWD_WAVES=1" -- --steps 20 --warmup 4 --micro-batch 32 | tee gpurun_out/ab_ln_waves_mb32.txt
bash scripts/abn.sh "LLMT_LN_BWD_WAVES=3" "LLMT_LN_BWD_WAVES=2" "LLMT_LN_BWD_WAVES=1" -- --steps 12 --warmup 3 | tee gpurun_out/ab_ln_waves_mb128.txt
