#!/bin/bash
# A/B: hipGraph-captured optimizer step vs eager at micro-batch 32 and 128 (same box)
set -o pipefail
out=gpurun_out/s41; mkdir -p $out
for r in 1 2; do
  for mb in 32 128; do
    for g in "" "--cuda-graph"; do
      timeout -k 10 240 python -u bench.py --micro-batch $mb --steps 20 --warmup 5 $g > $out/b_${mb}_${g:-eager}_$r.txt 2>&1 || exit 1
      echo "mb$mb ${g:-eager} r$r: $(tail -1 $out/b_${mb}_${g:-eager}_$r.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $out/ab.txt
    done
  done
done
