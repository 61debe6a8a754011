#!/usr/bin/env bash
# Re-entry verification on one MI355X: GPU test tier, smoke, bench at micro-batch 128 and 32.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_mb128.log 2>&1
tail -1 gpurun_out/bench_mb128.log
timeout -k 10 300 python bench.py --micro-batch 32 > gpurun_out/bench_mb32.log 2>&1
tail -1 gpurun_out/bench_mb32.log
