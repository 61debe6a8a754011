#!/usr/bin/env bash
# End-of-session evidence: GPU tier + smoke, bench mb 128 / 32, rocprofv3 kernel table at mb 128,
# 2-rank bench rehearsal (gloo, ranks sharing the GPU), val-loss parity.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
OUT=gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench_mb128.log 2>&1
tail -1 $OUT/bench_mb128.log | cut -c1-200
timeout -k 10 300 python bench.py --micro-batch 32 > $OUT/bench_mb32.log 2>&1
tail -1 $OUT/bench_mb32.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof -o run -- \
  python3 bench.py --gpus 1 --steps 6 --warmup 3 > $OUT/bench_prof.log 2>&1
db=$(find $OUT/prof -name "*.db" | head -1)
python3 scripts/rocpd_stats.py "$db" 3 40 > $OUT/kernel_stats_mb128.txt
rm -f "$db"
tail -3 $OUT/kernel_stats_mb128.txt
timeout -k 10 400 python bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 --micro-batch 32 > $OUT/bench_2rank_gloo.log 2>&1
tail -1 $OUT/bench_2rank_gloo.log | cut -c1-200
timeout -k 10 600 python -u bench/parity.py --steps 300 --micro-batch 32 > $OUT/parity.jsonl 2> $OUT/parity.err
tail -1 $OUT/parity.jsonl
