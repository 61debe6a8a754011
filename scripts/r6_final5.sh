#!/usr/bin/env bash
# Round 6 closing evidence after the LDS-DMA attention forward: full GPU suite, smoke, headline
# bench + kernel table, micro-batch 32, XL deterministic, gloo world 2, attention PMC rows
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6_final5}
bash scripts/gpu_session.sh -o "$OUT" tests smoke bench:128 prof:128 gloo2 || exit $?
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; tail -n 1 "$OUT/$name.log" | cut -c1-400; [ $rc -eq 0 ] || { echo "FAILED $name rc=$rc"; exit $rc; }; }
step bench_mb32 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --micro-batch 32
step bench_xl_det 400 python -u bench.py --gpus 1 --steps 10 --warmup 3 --model gpt2-xl --micro-batch 32 --grad-accum 2 --deterministic
mkdir -p "$OUT/pmc"
step pmc_attn 300 env OUT="$OUT/pmc" TAG=attn bash scripts/pmc_kernels.sh python3 bench/micro.py attn_ours 128 12
echo done
