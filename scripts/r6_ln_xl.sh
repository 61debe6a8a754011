#!/usr/bin/env bash
# Round 6: GPT-2 XL LayerNorm backward, split-row (release) vs whole-row lean kernel (variant)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6_ln_xl}
mkdir -p "$OUT"
V=llmtrain/ops/variants/_llmtrain_hip_lnlean.so
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; grep '^{' "$OUT/$name.log" | cut -c1-200; [ $rc -eq 0 ] || { tail -5 "$OUT/$name.log"; exit $rc; }; }
LLMTRAIN_HIP_EXT=$V step tests 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "layernorm or ln_"
for r in 1 2; do
  step micro_rel_$r 120 python -u bench/micro.py ln 32768 1600
  LLMTRAIN_HIP_EXT=$V step micro_lean_$r 120 python -u bench/micro.py ln 32768 1600
done
XL="--model gpt2-xl --micro-batch 32 --grad-accum 2 --deterministic --steps 6 --warmup 3"
for r in 1 2; do
  step xl_rel_$r 400 python -u bench.py --gpus 1 $XL
  LLMTRAIN_HIP_EXT=$V step xl_lean_$r 400 python -u bench.py --gpus 1 $XL
done
echo done
