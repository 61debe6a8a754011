#!/usr/bin/env bash
# Row-chunked LM head: GPU tests, then same-box A/B in the bench (mb 128 and 32).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/hc
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash scripts/abn.sh "LLMTRAIN_HEAD_CHUNK_ROWS=0" "LLMTRAIN_HEAD_CHUNK_ROWS=-1" "LLMTRAIN_HEAD_CHUNK_ROWS=32768" -- --steps 15 --warmup 4 > $OUT/ab128.txt 2>&1
cat $OUT/ab128.txt
bash scripts/abn.sh "LLMTRAIN_HEAD_CHUNK_ROWS=0" "LLMTRAIN_HEAD_CHUNK_ROWS=-1" -- --steps 15 --warmup 4 --micro-batch 32 > $OUT/ab32.txt 2>&1
cat $OUT/ab32.txt
