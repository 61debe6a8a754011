#!/usr/bin/env bash
# Tune every hipBLASLt/rocBLAS GEMM the bench issues with PyTorch TunableOp, starting from the
# shipped table (llmtrain/runtime/tuned/), then (AB=1) A/B the bench with and without the table on
# the same box.  New table: gpurun_out/tunableop/tuned0.csv (the shipped rows + the new shapes).
#   BENCH_ARGS="--model gpt2-xl --micro-batch 16 --grad-accum 2" AB=0 bash scripts/tune_gemms.sh
# FRESH=1: re-tune every shape from an empty table, and A/B it against the shipped table instead
# of the library heuristics (e.g. with PYTORCH_TUNABLEOP_ROTATING_BUFFER_SIZE=1024, so candidates
# are timed on operands that are not cache-resident, as in the step).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/tunableop
mkdir -p "$OUT"
MB=${MB:-128}
if [ "${FRESH:-0}" = 1 ]; then rm -f "$OUT/tuned0.csv"; else cp llmtrain/runtime/tuned/gemm_tunableop_gfx950.csv "$OUT/tuned0.csv"; fi
# a heartbeat on stdout while the tuning pass runs (it prints nothing for minutes at a time)
( while sleep 50; do echo "tuning... $(wc -l < "$OUT/tune.log" 2>/dev/null || echo 0) log lines"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
# 1) tuning pass: every (op, shape) not yet in the table is benchmarked over all library solutions
#    (TunableOp inserts the device ordinal into a file name without one: tuned.csv -> tuned0.csv)
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=${VERBOSE:-1} \
PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=${TUNE_ITERS:-30} \
PYTORCH_TUNABLEOP_FILENAME="$OUT/tuned%d.csv" \
  timeout -k 10 ${TUNE_LIMIT:-900} python bench.py --steps 1 --warmup 1 --micro-batch "$MB" ${BENCH_ARGS:-} \
  > "$OUT/tune.log" 2>&1 || { echo "tuning failed"; tail -30 "$OUT/tune.log"; exit 1; }
kill $HB 2>/dev/null || true
cat "$OUT"/tuned0.csv
[ "${AB:-1}" = 1 ] || exit 0
# 2) same-box A/B: library heuristics vs the tuned table (tuning off, look-ups only)
for round in 1 2; do
  for tag in base tuned; do
    if [ "$tag" = tuned ]; then envs="PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$OUT/tuned%d.csv"
    elif [ "${FRESH:-0}" = 1 ]; then envs="LLMTRAIN_TUNED_GEMMS=1"; else envs="LLMTRAIN_TUNED_GEMMS=0"; fi
    env -u PYTORCH_TUNABLEOP_ROTATING_BUFFER_SIZE $envs timeout -k 10 300 python bench.py --steps 20 --warmup 5 --micro-batch "$MB" ${BENCH_ARGS:-} \
      > "$OUT/bench_${tag}_${round}.log" 2>&1 || { echo "bench $tag failed"; tail -20 "$OUT/bench_${tag}_${round}.log"; exit 1; }
    echo "$tag round$round: $(tail -1 "$OUT/bench_${tag}_${round}.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
