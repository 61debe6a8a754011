#!/usr/bin/env bash
# Round 6 session 2: full GPU suite on the new defaults, kernel table, parity seeds 1/2, XL A/B
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6_s2
mkdir -p "$OUT"
bash scripts/gpu_session.sh -o "$OUT" tests prof:128 || exit $?
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; tail -n 2 "$OUT/$name.log"; [ $rc -eq 0 ] || { echo "FAILED $name rc=$rc"; exit $rc; }; }
step parity_s12 900 python -u bench/parity.py --steps 1500 --micro-batch 16 --seeds 1,2 --paths fused:fp32,fused:bf16
for r in bf16 fp32; do
  step "xl_det_$r" 400 python -u bench.py --gpus 1 --steps 10 --warmup 3 --model gpt2-xl --micro-batch 32 --grad-accum 2 --deterministic --residual $r
done
echo done
