# one-stream schedule: which GEMMs should run on the hand-written fused kernel at M = 131072
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/s15
bash scripts/abn.sh "LLMTRAIN_FGEMM_ANY=dx_gelu,dx_attn" "LLMTRAIN_FGEMM_ANY=dx_attn" "LLMTRAIN_FGEMM_ANY=dx_gelu,dx_attn,fwd_gelu" "LLMTRAIN_FGEMM_ANY=dx_gelu,dx_attn,fwd_gelu,fwd,dx" -- --steps 20 --warmup 5 > gpurun_out/s15/ab_fgemm_mb128.txt 2>&1 || exit 1
cat gpurun_out/s15/ab_fgemm_mb128.txt
