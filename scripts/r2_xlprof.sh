#!/usr/bin/env bash
# GPT-2 XL kernel table (rocprofv3 kernel trace, mb 16 x grad-accum 2).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/xlprof
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format rocpd -d "$OUT" -o run -- \
  python3 bench.py --model gpt2-xl --micro-batch 16 --grad-accum 2 --steps 4 --warmup 2 > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log" | cut -c1-200
db=$(find "$OUT" -name "*.db" | head -1)
python3 scripts/rocpd_stats.py "$db" 2 40 > "$OUT/kernel_stats_xl.txt"
rm -f "$db"
head -30 "$OUT/kernel_stats_xl.txt"
tail -4 "$OUT/kernel_stats_xl.txt"
