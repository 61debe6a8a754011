# same-box step A/B of the weight-gradient kernels + counter passes on the ping-pong kernel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/s3
OUT=gpurun_out/s3 TAG=pp_qkv bash scripts/pmc_kernels.sh python3 bench/wgrad_pp.py one --gemm qkv --variant pp --reps 10 > gpurun_out/s3/pmc_pp.txt 2>&1 || exit 1
OUT=gpurun_out/s3 TAG=r3_qkv bash scripts/pmc_kernels.sh python3 bench/wgrad_pp.py one --gemm qkv --variant r3_tile256 --reps 10 > gpurun_out/s3/pmc_r3.txt 2>&1 || exit 1
bash scripts/abn.sh "LLMTRAIN_WGRAD_KERNEL=r3" "LLMTRAIN_WGRAD_KERNEL=pp" -- --steps 20 --warmup 5 > gpurun_out/s3/ab_mb128.txt 2>&1 || exit 1
bash scripts/abn.sh "LLMTRAIN_WGRAD_KERNEL=r3" "LLMTRAIN_WGRAD_KERNEL=pp" -- --steps 30 --warmup 5 --micro-batch 32 > gpurun_out/s3/ab_mb32.txt 2>&1 || exit 1
cat gpurun_out/s3/ab_mb128.txt gpurun_out/s3/ab_mb32.txt
