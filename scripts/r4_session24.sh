#!/bin/bash
# micro-batch 32: tune the fc forward on the library (fused GELU epilogue bypassed), install the
# table on this box, then A/B fused fc+GELU vs library fc + GELU pass
set -eo pipefail
O=gpurun_out/s24
mkdir -p $O
LLMTRAIN_FGEMM_NEVER=fwd,fwd_gelu MB=32 AB=0 TUNE_LIMIT=600 bash scripts/tune_gemms.sh > $O/tune.txt 2>&1
grep "_32768_" gpurun_out/tunableop/tuned0.csv > $O/rows_32768.csv
cp gpurun_out/tunableop/tuned0.csv llmtrain/runtime/tuned/gemm_tunableop_gfx950.csv
bash scripts/abn.sh "LLMTRAIN_FGEMM_NEVER=" "LLMTRAIN_FGEMM_NEVER=fwd_gelu" -- --micro-batch 32 --steps 20 --warmup 5 > $O/ab_fc_fwd_mb32.txt 2>&1
