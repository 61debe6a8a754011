#!/usr/bin/env bash
# mb 128: attention out-projection dX with the delta / V-bias epilogue at any size, and the
# attention backward's fused delta, vs the default (hipBLASLt dX + delta kernel).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/abn.sh "X=0" "LLMTRAIN_FGEMM_ANY_SIZE=dx_gelu,dx_attn" "LLMT_ATTN_FUSED_DELTA=1" -- --steps 12 --warmup 3 | tee gpurun_out/ab_attn_dx_mb128.txt
