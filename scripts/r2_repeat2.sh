#!/usr/bin/env bash
# Bitwise repeatability of the hand-written kernels with a concurrent GEMM stream (timing noise).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/det
export TMPDIR=/tmp
NOISE=1 timeout -k 10 400 python bench/repeat_check.py 32768 10 2>/dev/null | tee gpurun_out/det/repeat_32k_noise.jsonl
