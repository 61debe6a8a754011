#!/usr/bin/env bash
# Is the deterministic fused path (run.deterministic, the parity harness's default) bitwise
# reproducible at GPT-2 124M / mb 32?  Two runs per variant, 100 steps each.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/det
export TMPDIR=/tmp
for v in "X=0" "LLMTRAIN_TUNED_GEMMS=0" "LLMTRAIN_WGRAD_STREAM=0" "LLMTRAIN_FUSED_GEMM=0"; do
  for r in 1 2; do
    env $v timeout -k 10 300 python -u bench/parity.py --steps 100 --micro-batch 32 --paths fused \
      > gpurun_out/det/run.jsonl 2> gpurun_out/det/run.err
    echo "[$v] r$r $(grep '"path"' gpurun_out/det/run.jsonl)" | tee -a gpurun_out/det/runs.txt
  done
done
