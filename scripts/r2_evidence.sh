#!/usr/bin/env bash
# Evidence pass: full GPU tier + smoke, rocprofv3 kernel tables at micro-batch 128 / 32, val-loss parity.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
tail -1 gpurun_out/smoke.log
bash scripts/r2_prof.sh
timeout -k 10 600 python -u bench/parity.py --steps 300 --micro-batch 32 > gpurun_out/parity.jsonl 2> gpurun_out/parity.err
tail -1 gpurun_out/parity.jsonl
