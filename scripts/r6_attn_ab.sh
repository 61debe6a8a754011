#!/usr/bin/env bash
# Round 6: attention-backward variants (llmtrain/ops/variants/) — numerics, then interleaved timing
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6_attn_ab
mkdir -p "$OUT"
VARIANTS=${VARIANTS:-"rcinit prio both"}
ext() { [ "$1" = release ] && echo "" || echo "llmtrain/ops/variants/_llmtrain_hip_$1.so"; }
for v in $VARIANTS; do
  echo "== tests $v"
  LLMTRAIN_HIP_EXT=$(ext $v) timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests_$v.log" 2>&1 || { tail -20 "$OUT/tests_$v.log"; exit 1; }
  tail -1 "$OUT/tests_$v.log"
done
for round in 1 2; do
  for v in release $VARIANTS; do
    echo "== time $v round $round"
    LLMTRAIN_HIP_EXT=$(ext $v) timeout -k 10 200 python -u bench/micro.py attn_ours 128 12 >> "$OUT/time_$v.jsonl" 2>> "$OUT/time_$v.err" || exit 1
    LLMTRAIN_HIP_EXT=$(ext $v) timeout -k 10 200 python -u bench/micro.py attn_ours 32 25 >> "$OUT/time_$v.jsonl" 2>> "$OUT/time_$v.err" || exit 1
    tail -6 "$OUT/time_$v.jsonl"
  done
done
