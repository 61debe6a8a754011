#!/usr/bin/env bash
# Round 3, first GPU session: GPU tests, deterministic-mode probe (side stream on / off), and a
# 2-rank gloo-on-one-GPU rehearsal of the bucket timeline.  Each GPU step has its own limit.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3a; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 240 python -u bench/determinism_probe.py --steps 150 --reps 3 > $O/det_side.jsonl 2> $O/det_side.err; rc=$?
echo "det_side rc=$rc"; tail -2 $O/det_side.jsonl
[ $rc -le 1 ] || exit 1
LLMTRAIN_WGRAD_STREAM=0 timeout -k 10 240 python -u bench/determinism_probe.py --steps 150 --reps 3 > $O/det_noside.jsonl 2> $O/det_noside.err; rc=$?
echo "det_noside rc=$rc"; tail -1 $O/det_noside.jsonl
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --steps 4 --warmup 2 --micro-batch 16 > $O/bench_2rank_gloo.log 2>&1; rc=$?
echo "gloo2 rc=$rc"; tail -1 $O/bench_2rank_gloo.log
