#!/usr/bin/env bash
# Library GEMMs (hipBLASLt, shipped solution table) repeated with and without a concurrent GEMM stream.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/det
export TMPDIR=/tmp
LIB=1 timeout -k 10 300 python bench/repeat_check.py 32768 10 2>/dev/null | tee gpurun_out/det/repeat_lib_32k.jsonl
LIB=1 NOISE=1 timeout -k 10 300 python bench/repeat_check.py 32768 10 2>/dev/null | tee gpurun_out/det/repeat_lib_32k_noise.jsonl
