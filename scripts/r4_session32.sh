#!/bin/bash
# attention backward: dS^T image written from the packed bf16 dS (one conversion instead of two);
# numerics, then op time and step A/B against the previous build (LLMTRAIN_HIP_EXT)
set -eo pipefail
O=gpurun_out/s32
mkdir -p $O
OLD=$PWD/llmtrain/ops/_llmtrain_hip_old.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py tests/test_deterministic_gpu.py > $O/pytest.txt 2>&1
for r in 1 2; do
  LLMTRAIN_HIP_EXT=$OLD timeout -k 10 120 python -u bench/micro.py attn 128 2>&1 | grep "llmtrain bwd" | sed "s/^/old /" >> $O/attn.txt
  timeout -k 10 120 python -u bench/micro.py attn 128 2>&1 | grep "llmtrain bwd" | sed "s/^/new /" >> $O/attn.txt
done
bash scripts/abn.sh "LLMTRAIN_HIP_EXT=$OLD" "LLMTRAIN_HIP_EXT=" -- --steps 10 --warmup 3 > $O/ab_mb128.txt 2>&1
