#!/usr/bin/env bash
# Round 6: deterministic LM-head logits on the fixed-order kernel — GPU tests + same-box A/B
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6_det_head
mkdir -p "$OUT"
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; tail -n 2 "$OUT/$name.log"; [ $rc -eq 0 ] || { echo "FAILED $name rc=$rc"; exit $rc; }; }
step pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm_fused or deterministic"
for i in 1 2; do
  for arm in ours library; do
    step "mb32_${arm}_$i" 300 python -u bench/det_head_ab.py $arm --gpus 1 --steps 20 --warmup 5 --micro-batch 32 --deterministic
  done
done
for arm in ours library; do
  step "xl_${arm}" 400 python -u bench/det_head_ab.py $arm --gpus 1 --steps 10 --warmup 3 --model gpt2-xl --micro-batch 32 --grad-accum 2 --deterministic
done
echo done
