#!/usr/bin/env bash
# Round 6: ping-pong attention backward — numerics, op timing and step A/B against the
# attn_bwd_kernel sweep (variant build LLMT_ATTN_PINGPONG=0)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6_attn_pp}
mkdir -p "$OUT"
NOPP=llmtrain/ops/variants/_llmtrain_hip_nopp.so
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; tail -n 3 "$OUT/$name.log"; [ $rc -eq 0 ] || { echo "== $name FAILED rc=$rc"; exit $rc; }; }
step tests 400 python -u -m pytest tests/test_attention_gpu.py tests/test_deterministic_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
for r in 1 2; do
  step micro_pp_$r 200 python -u bench/micro.py attn_ours 128 12
  LLMTRAIN_HIP_EXT=$NOPP step micro_nopp_$r 200 python -u bench/micro.py attn_ours 128 12
done
for r in 1 2; do
  step bench_pp_$r 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --micro-batch 128
  LLMTRAIN_HIP_EXT=$NOPP step bench_nopp_$r 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --micro-batch 128
done
echo done
