#!/usr/bin/env bash
# solo micro-benchmarks at the micro-batch-128 shapes (M = 131072 tokens): LayerNorm / GELU
# bandwidth, fused-epilogue GEMMs vs hipBLASLt, attention forward probe
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/micro
mkdir -p $OUT
timeout -k 10 60 bench/native/bin/fwd_new_probe 32 probe > $OUT/probe.log 2>&1
grep -E "grid|mean" $OUT/probe.log
timeout -k 10 120 python bench/micro.py ln 131072 2>&1 | tee $OUT/ln.log | grep op
timeout -k 10 300 python bench/micro.py fgemm 131072 2>&1 | tee $OUT/fgemm.log | grep gemm
