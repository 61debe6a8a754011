#!/usr/bin/env bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/det
export TMPDIR=/tmp
for r in 1 2 3; do
  env ${DET_ENV:-X=0} timeout -k 10 300 python -u bench/parity.py --steps 300 --micro-batch 32 --paths fused \
    > gpurun_out/det/run.jsonl 2> gpurun_out/det/run.err
  echo "[300 steps] r$r $(grep '"path"' gpurun_out/det/run.jsonl)" | tee -a gpurun_out/det/runs300.txt
done
