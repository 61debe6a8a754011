#!/usr/bin/env bash
# Round 6: attention forward with K/V by LDS-DMA at 4 workgroups per CU (the release build) —
# the GPU suite on it, then step A/Bs against the register-staged kernel (variant build "fstage",
# the previous attention_fwd.hip)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6_fdma2}
mkdir -p "$OUT"
V=llmtrain/ops/variants/_llmtrain_hip_fstage.so
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; tail -n 3 "$OUT/$name.log"; [ $rc -eq 0 ] || { echo "== $name FAILED rc=$rc"; exit $rc; }; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
for r in 1 2; do
  step bench_dma_$r 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --micro-batch 128
  LLMTRAIN_HIP_EXT=$V step bench_stage_$r 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --micro-batch 128
done
step xl_dma 400 python -u bench.py --gpus 1 --model gpt2-xl --micro-batch 32 --grad-accum 2 --deterministic --steps 6 --warmup 2
LLMTRAIN_HIP_EXT=$V step xl_stage 400 python -u bench.py --gpus 1 --model gpt2-xl --micro-batch 32 --grad-accum 2 --deterministic --steps 6 --warmup 2
echo done
