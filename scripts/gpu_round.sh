#!/usr/bin/env bash
# One GPU-box session: kernel/engine tests, then a short bench. Every GPU step has its own
# time limit and the chain stops at the first failure (never retried).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-10}
WARMUP=${WARMUP:-3}
MB=${MB:-32}
timeout -k 10 600 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --gpus 1 --steps "$STEPS" --warmup "$WARMUP" --micro-batch "$MB" ${BENCH_ARGS:-} \
  > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench.log; exit 1; }
tail -3 gpurun_out/bench.log
