#!/usr/bin/env bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC counters in this run).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
mkdir -p "$OUT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 bench.py --gpus 1 --steps "${STEPS:-5}" --warmup "${WARMUP:-2}" --micro-batch "${MB:-32}" ${BENCH_ARGS:-} \
  > "$OUT/bench.log" 2>&1 || { echo "profile failed"; tail -30 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
find "$OUT" -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -30 "{}"'
