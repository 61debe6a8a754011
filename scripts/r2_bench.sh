#!/usr/bin/env bash
# bench at micro-batch 128 and 32 (20 timed steps each, no profiler) + one rocprofv3 kernel table
# at micro-batch 128
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r2bench
mkdir -p "$OUT"
for MB in 128 32; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --micro-batch $MB > "$OUT/bench_mb$MB.log" 2>&1
  tail -1 "$OUT/bench_mb$MB.log"
done
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d "$OUT/prof" -o run -- \
    python3 bench.py --gpus 1 --steps 6 --warmup 3 --micro-batch 128 > "$OUT/prof_bench.log" 2>&1
  db=$(find "$OUT/prof" -name "*.db" | head -1)
  python3 scripts/rocpd_stats.py "$db" 3 40 > "$OUT/kernel_stats_mb128.txt"
  rm -f "$db"
  head -16 "$OUT/kernel_stats_mb128.txt" | cut -c1-150
  tail -3 "$OUT/kernel_stats_mb128.txt"
fi
