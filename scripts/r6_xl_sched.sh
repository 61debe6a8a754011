#!/usr/bin/env bash
# Round 6: GPT-2 XL deterministic schedule A/B (serial vs ours), same box, alternating
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6_xl_sched}
mkdir -p "$OUT"
XL="--model gpt2-xl --micro-batch 32 --grad-accum 2 --deterministic --steps 6 --warmup 3"
for r in 1 2; do
  for s in serial ours; do
    echo "== $s $r"
    LLMTRAIN_DET_SCHEDULE=$s timeout -k 10 400 python -u bench.py --gpus 1 $XL > "$OUT/xl_${s}_$r.log" 2>&1 || { tail -5 "$OUT/xl_${s}_$r.log"; exit 1; }
    grep '^{' "$OUT/xl_${s}_$r.log" | cut -c1-200
  done
done
echo done
