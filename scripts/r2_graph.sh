#!/usr/bin/env bash
# hipGraph-captured optimizer steps: tests, then eager vs graph on the reference presets' shapes.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_graph_step_gpu.py tests/test_kernels_gpu.py -x -v \
  --timeout 180 --timeout-method thread -k "graph or adamw" > gpurun_out/graph_tests.log 2>&1 \
  || { echo "tests failed"; tail -60 gpurun_out/graph_tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/graph_tests.log | tail -8
for m in wikitext-ddp wikitext-better; do
  for g in "" "--cuda-graph"; do
    echo "$m $g: $(timeout -k 10 300 python bench.py --model $m --micro-batch 16 --steps 50 --warmup 5 $g 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'tok/s', d['ms_per_step'], 'ms/step')")"
  done
done
for g in "" "--cuda-graph"; do
  echo "124M mb32 $g: $(timeout -k 10 300 python bench.py --micro-batch 32 --steps 20 --warmup 4 $g 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'tok/s', d['ms_per_step'], 'ms/step')")"
done
