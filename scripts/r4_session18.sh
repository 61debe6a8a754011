#!/bin/bash
# 8-wave ping-pong attention forward: numerics (fp32 oracle tests), op timing vs the 4-wave kernel, step A/B
set -eo pipefail
O=gpurun_out/s18
mkdir -p $O
LLMT_ATTN_FWD_PP=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py > $O/pytest_attention.txt 2>&1
LLMT_ATTN_BWD_STAGGER=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py > $O/pytest_attention_stagger.txt 2>&1
for r in 1 2; do
  for sg in 0 1; do
    LLMT_ATTN_BWD_STAGGER=$sg timeout -k 10 120 python -u bench/micro.py attn 128 2>&1 | grep "llmtrain bwd" | sed "s/^/stagger$sg /" >> $O/attn_bwd.txt
  done
done
for r in 1 2; do
  for pp in 0 1; do
    LLMT_ATTN_FWD_PP=$pp timeout -k 10 120 python -u bench/micro.py attn 128 2>&1 | grep "llmtrain fwd" | sed "s/^/pp$pp /" >> $O/attn_fwd.txt
    LLMT_ATTN_FWD_PP=$pp timeout -k 10 120 python -u bench/micro.py attn 32 2>&1 | grep "llmtrain fwd" | sed "s/^/pp$pp B32 /" >> $O/attn_fwd.txt
  done
done
bash scripts/abn.sh "LLMT_ATTN_FWD_PP=0" "LLMT_ATTN_FWD_PP=1" "LLMT_ATTN_FWD_PP=1 LLMT_ATTN_BWD_STAGGER=1" -- --steps 10 --warmup 3 > $O/ab_attn_fwd_pp_mb128.txt 2>&1
