#!/usr/bin/env bash
# Fused-path val loss under kernel variants that must not change results (tiled GELU / AdamW: same
# per-element math) and one that reorders fp32 sums (LayerNorm-backward grid waves): a repeat shows
# the deterministic run reproduces bitwise.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pcheck
export TMPDIR=/tmp
for v in "X=0" "X=1" "LLMT_GELU_TILED=0 LLMT_ADAMW_TILED=0" "LLMT_LN_BWD_WAVES=3"; do
  env $v timeout -k 10 300 python -u bench/parity.py --steps 300 --micro-batch 32 --paths fused \
    > gpurun_out/pcheck/run.jsonl 2> gpurun_out/pcheck/run.err
  echo "[$v] $(grep '"path"' gpurun_out/pcheck/run.jsonl)" | tee -a gpurun_out/pcheck/variants.txt
done
