#!/usr/bin/env bash
# Round 6: MLP keeps gelu'(u) instead of u (model.extra.mlp_store) — numerics, step A/B, parity
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6_gd; mkdir -p "$OUT"
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; tail -n 1 "$OUT/$name.log" | cut -c1-330; [ $rc -eq 0 ] || { echo "FAILED $name rc=$rc"; tail -30 "$OUT/$name.log"; exit $rc; }; }
step pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm_fused or fused_matches or bench_shape"
for i in 1 2; do
  for m in u gd; do
    step "bench_${m}_$i" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --micro-batch 128 --mlp-store $m
  done
done
for m in u gd; do
  step "xl_${m}" 400 python -u bench.py --gpus 1 --steps 10 --warmup 3 --model gpt2-xl --micro-batch 32 --grad-accum 2 --deterministic --mlp-store $m
done
step parity 900 python -u bench/parity.py --steps 1500 --micro-batch 16 --seeds 1337,7,42 --paths fused:bf16:gd
echo done
