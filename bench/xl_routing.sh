#!/usr/bin/env bash
# GPT-2 XL (BASELINE config 5, micro-batch 16 x 4, the gpt2_xl_mi355x_ddp8 preset's shape until it moved to 32 x 2,
# run.deterministic) GEMM routing study on one GPU box:
#  1) a TunableOp pass with every forward / dX GEMM sent to the library (so each shape gets a
#     measured hipBLASLt / rocBLAS solution), table -> OUT/tuned_xl.csv;
#  2) with that table, a same-box interleaved A/B of the deterministic step: the default routing
#     (fused GEMM for A operands <= 64 MiB), every forward / dX GEMM on the library, and the
#     library for the plain forward GEMMs only (the fc forward keeps its fused bias + GELU).
#   bash bench/xl_routing.sh [OUT]
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/xl_routing}; mkdir -p "$OUT"
env LLMTRAIN_FGEMM_MAX_A_MB=0 LLMTRAIN_FGEMM_ANY=none MB=16 BENCH_ARGS="--model gpt2-xl --grad-accum 4" AB=0 \
  TUNE_LIMIT=900 timeout -k 10 1000 bash scripts/tune_gemms.sh > "$OUT/tune.log" 2>&1 \
  || { echo "tune failed"; tail -20 "$OUT/tune.log"; exit 1; }
tail -12 gpurun_out/tunableop/tuned0.csv
cp gpurun_out/tunableop/tuned0.csv "$OUT/tuned_xl.csv"
# the A/B below loads the box-tuned table in place of the shipped one; the shipped file is restored
# on exit, so a run in a working tree cannot leave the box's table behind to be committed
SHIPPED=llmtrain/runtime/tuned/gemm_tunableop_gfx950.csv
cp "$SHIPPED" "$OUT/shipped_table_backup.csv"
trap 'cp "$OUT/shipped_table_backup.csv" "$SHIPPED"' EXIT
cp gpurun_out/tunableop/tuned0.csv "$SHIPPED"
bash scripts/abn.sh "LLMTRAIN_FGEMM_MAX_A_MB=64" "LLMTRAIN_FGEMM_MAX_A_MB=0" "LLMTRAIN_FGEMM_NEVER=fwd" -- \
  --model gpt2-xl --micro-batch 16 --grad-accum 4 --deterministic --steps 4 --warmup 2 | tee "$OUT/ab_xl_det.txt"
