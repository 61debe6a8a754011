#!/usr/bin/env bash
# deterministic-mode round: determinism + attention/engine tests, full GPU tier, bench fast vs deterministic
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_deterministic_gpu.py tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest_det.log 2>&1 || { tail -50 $OUT/pytest_det.log; exit 1; }
tail -2 $OUT/pytest_det.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { grep -E "PASSED|FAILED|Error|error" $OUT/pytest_gpu.log | tail -30; tail -30 $OUT/pytest_gpu.log; exit 1; }
grep -E "resume:|worst" $OUT/pytest_gpu.log | head -20
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_mb128.log 2>&1
tail -1 $OUT/bench_mb128.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --deterministic > $OUT/bench_mb128_det.log 2>&1
tail -1 $OUT/bench_mb128_det.log
