#!/usr/bin/env bash
# Refresh side numbers: GPT-2 XL (mb16 x accum 2), GPT-2 124M at dropout 0.1, deterministic mode.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --model gpt2-xl --micro-batch 16 --grad-accum 2 --steps 6 --warmup 2 > gpurun_out/bench_xl.log 2>&1
tail -1 gpurun_out/bench_xl.log
timeout -k 10 300 python bench.py --dropout 0.1 > gpurun_out/bench_drop.log 2>&1
tail -1 gpurun_out/bench_drop.log
timeout -k 10 300 python bench.py --deterministic > gpurun_out/bench_det.log 2>&1
tail -1 gpurun_out/bench_det.log
bash scripts/abn.sh "LLMTRAIN_WGRAD_STREAM=1" "LLMTRAIN_WGRAD_STREAM=0" -- --steps 15 --warmup 4 | tee gpurun_out/ab_wgrad_stream_mb128.txt
bash scripts/abn.sh "LLMTRAIN_WGRAD_STREAM=1" "LLMTRAIN_WGRAD_STREAM=0" -- --steps 20 --warmup 4 --micro-batch 32 | tee gpurun_out/ab_wgrad_stream_mb32.txt
