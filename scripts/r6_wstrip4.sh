#!/usr/bin/env bash
# Round 6: weight-gradient tail tiling — op timing with the rounds planner, tests, XL step A/B
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6_wstrip4}
mkdir -p "$OUT"
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; tail -n 2 "$OUT/$name.log"; [ $rc -eq 0 ] || { echo "== $name FAILED rc=$rc"; exit $rc; }; }
step tests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_deterministic_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wgrad"
step time_xl 300 python -u bench/wgrad_pp.py time --model gpt2-xl --tokens 32768 --only pp_slab,pp_slab_square,pp_slab_bias,pp_slab_bias_square --rounds 3
XL="--model gpt2-xl --micro-batch 32 --grad-accum 2 --deterministic --steps 6 --warmup 3"
for i in 1 2; do
  step xl_tails_$i 400 python -u bench/wgrad_tail_ab.py tails --gpus 1 $XL
  step xl_square_$i 400 python -u bench/wgrad_tail_ab.py square --gpus 1 $XL
done
echo done
