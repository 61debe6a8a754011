#!/usr/bin/env bash
# Round 6: packed-fp32 (SLP) A/B: release vs -fno-slp-vectorize vs that + scalar attention-forward softmax
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6_slp}
mkdir -p "$OUT"
ext() { [ "$1" = rel ] && echo "" || echo "llmtrain/ops/variants/_llmtrain_hip_$1.so"; }
for v in noslp fwdscalar; do
  LLMTRAIN_HIP_EXT=$(ext $v) timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/tests_$v.log" 2>&1 || { tail -20 "$OUT/tests_$v.log"; exit 1; }
  echo "tests $v: $(tail -1 "$OUT/tests_$v.log")"
done
for r in 1 2; do
  for v in rel noslp fwdscalar; do
    LLMTRAIN_HIP_EXT=$(ext $v) timeout -k 10 200 python -u bench/micro.py attn_ours 128 12 2>/dev/null | sed "s/^{/{\"build\": \"$v\", /" >> "$OUT/micro.jsonl" || exit 1
  done
done
grep -h "fwd\|delta ready" "$OUT/micro.jsonl" | cut -c1-160
for r in 1 2; do
  for v in rel noslp fwdscalar; do
    LLMTRAIN_HIP_EXT=$(ext $v) timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --micro-batch 128 > "$OUT/bench_${v}_$r.log" 2>&1 || exit 1
    echo "bench $v $r: $(grep -o '"value": [0-9.]*' "$OUT/bench_${v}_$r.log")"
  done
done
echo done
