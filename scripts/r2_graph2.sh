#!/usr/bin/env bash
# Graph-captured steps with dropout: full GPU tier, then eager vs graph on the reference presets' shapes.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for m in wikitext-ddp wikitext-better; do
  for g in "" "--cuda-graph"; do
    echo "$m dropout0.1 $g: $(timeout -k 10 300 python bench.py --model $m --micro-batch 16 --dropout 0.1 --steps 50 --warmup 5 $g 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'tok/s', d['ms_per_step'], 'ms/step')")"
  done
done
