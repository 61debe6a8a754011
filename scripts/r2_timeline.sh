#!/usr/bin/env bash
# Kernel trace of the bench (micro-batch 128): per-step summary + one step's timeline.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/tl}
MB=${MB:-128}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d "$OUT/db" -o run -- \
  python3 bench.py --gpus 1 --steps 6 --warmup 3 --micro-batch $MB "$@" > "$OUT/bench.log" 2>&1
db=$(find "$OUT/db" -name "*.db" | head -1)
python3 scripts/rocpd_stats.py "$db" 3 45 > "$OUT/kernel_stats.txt"
python3 scripts/rocpd_timeline.py "$db" 5 > "$OUT/timeline.txt"
rm -f "$db"
tail -1 "$OUT/bench.log"; tail -3 "$OUT/kernel_stats.txt"; tail -5 "$OUT/timeline.txt"
