#!/usr/bin/env bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_graph_step_gpu.py -x -v --timeout 180 --timeout-method thread \
  > gpurun_out/graph3.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/graph3.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/graph3.log | tail -8
