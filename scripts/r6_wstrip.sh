#!/usr/bin/env bash
# Round 6: d = 1600 weight-gradient tiling (strips / swapped operands) — tests, numerics, timing A/B
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6_wstrip}
mkdir -p "$OUT"
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; tail -n 4 "$OUT/$name.log"; [ $rc -eq 0 ] || { echo "== $name FAILED rc=$rc"; exit $rc; }; }
step tests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_deterministic_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wgrad"
step check 300 python -u bench/wgrad_pp.py check
step time_xl 300 python -u bench/wgrad_pp.py time --model gpt2-xl --tokens 32768 --only pp_slab,pp_slab_square,pp_slab_bias,pp_slab_bias_square,pp_auto
step time_xl2 300 python -u bench/wgrad_pp.py time --model gpt2-xl --tokens 32768 --only pp_slab_square,pp_slab,pp_slab_bias_square,pp_slab_bias
step time_124m 300 python -u bench/wgrad_pp.py time --model gpt2-124m --tokens 131072 --only pp_auto,pp_slab_square
echo done
