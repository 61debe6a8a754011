#!/usr/bin/env bash
# Bitwise repeatability of the hand-written kernels (deterministic mode) at mb 32 / mb 128 shapes,
# then the 300-step deterministic run without the side stream (3x).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/det
export TMPDIR=/tmp
timeout -k 10 300 python bench/repeat_check.py 32768 6 2>/dev/null | tee gpurun_out/det/repeat_32k.jsonl
timeout -k 10 300 python bench/repeat_check.py 131072 4 2>/dev/null | tee gpurun_out/det/repeat_128k.jsonl
DET_ENV=LLMTRAIN_WGRAD_STREAM=0 bash scripts/r2_determinism300.sh
