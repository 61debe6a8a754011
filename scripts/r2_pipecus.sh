#!/usr/bin/env bash
# Side-stream weight gradients on the software-pipelined 512-register kernel with the split planned
# for fewer CUs (the rest stay free for the main stream's kernels) vs the default 336-register kernel.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/abn.sh "X=0" "LLMT_WGRAD_PIPE=4" "LLMT_WGRAD_PIPE=4 LLMT_WGRAD_CUS=192" "LLMT_WGRAD_PIPE=4 LLMT_WGRAD_CUS=224" "LLMT_WGRAD_CUS=192" -- --steps 12 --warmup 3 | tee gpurun_out/ab_pipe_cus_mb128.txt
