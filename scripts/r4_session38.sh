#!/bin/bash
# deterministic mode: LM-head dX on our kernel (the library's deep-reduction solution varied run to run)
set -eo pipefail
O=gpurun_out/s38
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_deterministic_gpu.py > $O/pytest_det.txt 2>&1
timeout -k 10 400 python -u bench/determinism_probe.py --steps 80 --reps 3 --micro-batch 8 > $O/probe_mb8.jsonl 2> $O/probe_mb8.err || [ $? -eq 1 ]
timeout -k 10 400 python -u bench/determinism_probe.py --steps 60 --reps 3 --micro-batch 32 > $O/probe_mb32.jsonl 2> $O/probe_mb32.err || [ $? -eq 1 ]
for r in 1 2; do
  for mb in 32 128; do
    for flag in "" "--deterministic"; do
      v=$(timeout -k 10 300 python bench.py --micro-batch $mb --steps 15 --warmup 4 $flag 2>/dev/null | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
      echo "[mb$mb ${flag:-fast}] round$r: $v tok/s" >> $O/ab_det.txt
    done
  done
done
