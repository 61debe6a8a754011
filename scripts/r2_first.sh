set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r2a
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r2a/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r2a/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2a/bench_mb128.log 2>&1
tail -1 gpurun_out/r2a/bench_mb128.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --micro-batch 32 > gpurun_out/r2a/bench_mb32.log 2>&1
tail -1 gpurun_out/r2a/bench_mb32.log
