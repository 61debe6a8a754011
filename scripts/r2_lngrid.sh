#!/usr/bin/env bash
# LayerNorm backward grid cap: 256 workgroups (one column-sum pass) vs the occupancy-sized grid.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LLMT_LN_BWD_MAXGRID=256 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k layernorm > gpurun_out/lngrid_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/lngrid_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/lngrid_tests.log)"
bash scripts/abn.sh "LLMT_LN_BWD_MAXGRID=0" "LLMT_LN_BWD_MAXGRID=256" "LLMT_LN_BWD_MAXGRID=512" -- --steps 20 --warmup 4 --micro-batch 32 | tee gpurun_out/ab_ln_grid_mb32.txt
bash scripts/abn.sh "LLMT_LN_BWD_MAXGRID=0" "LLMT_LN_BWD_MAXGRID=256" -- --model gpt2-xl --micro-batch 16 --grad-accum 2 --steps 6 --warmup 2 | tee gpurun_out/ab_ln_grid_xl.txt
