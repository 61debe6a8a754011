# one stream vs the weight-gradient side stream (fast mode), fills with one stream, kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/s12
bash scripts/abn.sh "LLMTRAIN_WGRAD_STREAM=1" "LLMTRAIN_WGRAD_STREAM=0" "LLMTRAIN_WGRAD_STREAM=0 LLMT_WPP_FILL=0" -- --steps 20 --warmup 5 > gpurun_out/s12/ab_stream_mb128.txt 2>&1 || exit 1
bash scripts/abn.sh "LLMTRAIN_WGRAD_STREAM=1" "LLMTRAIN_WGRAD_STREAM=0" "LLMTRAIN_WGRAD_STREAM=0 LLMT_WPP_FILL=0" -- --steps 30 --warmup 5 --micro-batch 32 > gpurun_out/s12/ab_stream_mb32.txt 2>&1 || exit 1
cat gpurun_out/s12/ab_stream_mb128.txt gpurun_out/s12/ab_stream_mb32.txt
LLMTRAIN_WGRAD_STREAM=0 bash scripts/gpu_session.sh -o gpurun_out/s12 prof:128 > gpurun_out/s12/prof.log 2>&1 || exit 1
head -30 gpurun_out/s12/kernel_stats_mb128.txt
tail -4 gpurun_out/s12/kernel_stats_mb128.txt
