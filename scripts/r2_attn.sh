#!/usr/bin/env bash
# attention coverage round: new attention/engine GPU tests, the full GPU tier, a short bench
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2b
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_attention_gpu.py tests/test_engine_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r2b/pytest_attn.log 2>&1 || { tail -60 gpurun_out/r2b/pytest_attn.log; exit 1; }
tail -3 gpurun_out/r2b/pytest_attn.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2b/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r2b/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r2b/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2b/bench_mb128.log 2>&1
tail -1 gpurun_out/r2b/bench_mb128.log
