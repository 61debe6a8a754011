# step A/B: weight-gradient fills LDS-DMA (128 KiB ring) vs register-staged (64 KiB), then a kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/s10
bash scripts/abn.sh "LLMT_WPP_FILL=0" "LLMT_WPP_FILL=1 LLMT_WPP_SLOTS=2" -- --steps 20 --warmup 5 > gpurun_out/s10/ab_fill_mb128.txt 2>&1 || exit 1
bash scripts/abn.sh "LLMT_WPP_FILL=0" "LLMT_WPP_FILL=1 LLMT_WPP_SLOTS=2" -- --steps 30 --warmup 5 --micro-batch 32 > gpurun_out/s10/ab_fill_mb32.txt 2>&1 || exit 1
cat gpurun_out/s10/ab_fill_mb128.txt gpurun_out/s10/ab_fill_mb32.txt
bash scripts/gpu_session.sh -o gpurun_out/s10 prof:128 > gpurun_out/s10/prof.log 2>&1 || exit 1
head -45 gpurun_out/s10/kernel_stats_mb128.txt
