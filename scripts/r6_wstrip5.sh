#!/usr/bin/env bash
# Round 6: weight-gradient tail tiling — full GPU suite, XL step A/B (final planner), XL kernel table
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6_wstrip5}
mkdir -p "$OUT"
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; tail -n 2 "$OUT/$name.log"; [ $rc -eq 0 ] || { echo "== $name FAILED rc=$rc"; exit $rc; }; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
XL="--model gpt2-xl --micro-batch 32 --grad-accum 2 --deterministic --steps 6 --warmup 3"
for i in 1 2; do
  step xl_square_$i 400 python -u bench/wgrad_tail_ab.py square --gpus 1 $XL
  step xl_tails_$i 400 python -u bench/wgrad_tail_ab.py tails --gpus 1 $XL
done
PROF_TAG=xl bash scripts/gpu_session.sh -o "$OUT" prof:32:--model,gpt2-xl,--grad-accum,2,--deterministic || exit 1
echo done
