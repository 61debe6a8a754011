# weight-gradient split-K epilogue in the step: slabs + finishing launch vs fp32 atomics (fast mode)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/s11
timeout -k 10 200 python -u bench/wgrad_pp.py check > gpurun_out/s11/check_default.log 2>&1; echo "check rc=$?"; grep -c '"ok": false' gpurun_out/s11/check_default.log
LLMT_WPP_EPI=atomic timeout -k 10 120 python -u bench/wgrad_pp.py time --tokens 131072 --only pp_auto,pp_slab_bias > gpurun_out/s11/time_atomic.log 2>&1
bash scripts/abn.sh "LLMT_WPP_EPI=slab" "LLMT_WPP_EPI=atomic" -- --steps 20 --warmup 5 > gpurun_out/s11/ab_epi_mb128.txt 2>&1 || exit 1
bash scripts/abn.sh "LLMT_WPP_EPI=slab" "LLMT_WPP_EPI=atomic" -- --steps 30 --warmup 5 --micro-batch 32 > gpurun_out/s11/ab_epi_mb32.txt 2>&1 || exit 1
cat gpurun_out/s11/ab_epi_mb128.txt gpurun_out/s11/ab_epi_mb32.txt
bash scripts/abn.sh "LLMTRAIN_DET_SCHEDULE=serial" "LLMTRAIN_DET_SCHEDULE=ours" -- --steps 20 --warmup 5 --deterministic > gpurun_out/s11/ab_det_mb128.txt 2>&1 || exit 1
bash scripts/abn.sh "LLMTRAIN_DET_SCHEDULE=serial" "LLMTRAIN_DET_SCHEDULE=ours" -- --steps 30 --warmup 5 --micro-batch 32 --deterministic > gpurun_out/s11/ab_det_mb32.txt 2>&1 || exit 1
cat gpurun_out/s11/ab_det_mb128.txt gpurun_out/s11/ab_det_mb32.txt
