#!/usr/bin/env bash
# Round 6: fused GEMM, 4-wave / two-workgroups-per-CU shape — numerics, then timing vs 8-wave
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6_fgemm4; mkdir -p "$OUT"
echo "== tests"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm_fused" > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
echo "== timing 124M shapes"
timeout -k 10 300 python -u bench/micro.py fgemm_waves 131072 > "$OUT/waves_m131k.jsonl" 2>&1 || { tail "$OUT/waves_m131k.jsonl"; exit 1; }
cat "$OUT/waves_m131k.jsonl" | grep '^{'
echo "== timing XL shapes"
for shape in "1600 6400 2 1" "1600 6400 1 0" "1600 1600 3 1" "1600 4800 0 0" "6400 1600 0 1"; do
  for w in 8 4; do
    timeout -k 10 120 python -u bench/micro.py fgemm1 $shape 32768 $w >> "$OUT/waves_xl.jsonl" 2>&1 || exit 1
  done
done
grep '^{' "$OUT/waves_xl.jsonl"
