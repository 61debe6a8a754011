#!/usr/bin/env bash
# Weight-gradient kernel A/B at micro-batch-128 shapes (LLMT_WGRAD_PIPE variants), numerics first.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/wgab
for v in 4 5; do
  LLMT_WGRAD_PIPE=$v timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k wgrad tests/test_deterministic_gpu.py > gpurun_out/wgab/pytest$v.log 2>&1
done
for sh in "2304 768" "768 768" "3072 768" "768 3072"; do
  for v in ${VARIANTS:-0 4 5}; do
    echo -n "pipe=$v " >> gpurun_out/wgab/t.log
    LLMT_WGRAD_PIPE=$v timeout -k 10 60 python bench/wgrad_one.py $sh 131072 10 2>/dev/null >> gpurun_out/wgab/t.log
  done
done
