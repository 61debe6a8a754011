#!/usr/bin/env bash
# Round-2 profile pass: rocprofv3 kernel trace (SQLite) of the bench at micro-batch 128 and 32,
# summarised per step by scripts/rocpd_stats.py, plus the attention micro-benchmark.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r2prof
mkdir -p "$OUT"
for MB in 128 32; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d "$OUT/mb$MB" -o run -- \
    python3 bench.py --gpus 1 --steps 6 --warmup 3 --micro-batch $MB > "$OUT/bench_mb$MB.log" 2>&1
  tail -1 "$OUT/bench_mb$MB.log"
  db=$(find "$OUT/mb$MB" -name "*.db" | head -1)
  python3 scripts/rocpd_stats.py "$db" 3 40 > "$OUT/kernel_stats_mb$MB.txt"
  rm -f "$db"
  tail -4 "$OUT/kernel_stats_mb$MB.txt"
done
timeout -k 10 120 python3 bench/micro.py attn 128 > "$OUT/micro_attn_b128.log" 2>&1
cat "$OUT/micro_attn_b128.log"
