#!/usr/bin/env bash
# Round 6: how much of each fused-GEMM call is its epilogue (variant build without epilogues)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6_epi_probe; mkdir -p "$OUT"
for round in 1 2; do
  for v in release epiprobe; do
    ext=""; [ $v = epiprobe ] && ext=llmtrain/ops/variants/_llmtrain_hip_epiprobe.so
    for shape in "768 3072 2 1 131072" "768 3072 0 1 131072" "768 3072 1 0 131072" "768 3072 0 0 131072" "3072 768 0 1 131072" "1600 6400 2 1 32768" "1600 6400 1 0 32768" "6400 1600 0 1 32768"; do
      set -- $shape
      echo "$v $shape" >> "$OUT/probe_$v.jsonl"
      LLMTRAIN_HIP_EXT=$ext timeout -k 10 120 python -u bench/micro.py fgemm1 $1 $2 $3 $4 $5 >> "$OUT/probe_$v.jsonl" 2>> "$OUT/err.log" || { echo "fail $v $shape"; tail -5 "$OUT/err.log"; exit 1; }
    done
    tail -9 "$OUT/probe_$v.jsonl"
  done
done
