#!/usr/bin/env bash
# HBM bytes of the bandwidth-bound kernels (LayerNorm fwd/bwd, GELU, cross-entropy) at 128K tokens:
# one counter pass for FETCH_SIZE and one for WRITE_SIZE (TCC limits), kernel trace for durations.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcmem
mkdir -p "$OUT"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/$c" -o pmc -- \
    python3 bench/micro.py ln 131072 > "$OUT/$c.log" 2>&1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/${c}_ce" -o pmc -- \
    python3 bench/ce_one.py 131072 > "$OUT/${c}_ce.log" 2>&1
  echo "pass $c done"
done
find "$OUT" -name "*.csv" | head -20
