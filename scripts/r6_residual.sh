#!/usr/bin/env bash
# Round 6: bf16 residual-stream options — numerics, same-box step A/B, 1500-step parity (3 seeds)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6_residual
mkdir -p "$OUT"
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; tail -n 2 "$OUT/$name.log"; [ $rc -eq 0 ] || { echo "FAILED $name rc=$rc"; exit $rc; }; }
step pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "layernorm or embedding or fused_matches or bench_shape or sumsq"
for i in 1 2; do
  for r in fp32 bf16_grad bf16; do
    step "bench_${r}_$i" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --micro-batch 128 --residual $r
  done
done
if [ "${PARITY:-1}" = 1 ]; then
  step parity 1500 python -u bench/parity.py --steps 1500 --micro-batch 16 --seeds 1337,7,42 --paths fused,fused:bf16_grad,fused:bf16
fi
echo done
