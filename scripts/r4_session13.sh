# full GPU tier + smoke + headline benches with the round-4 defaults (one stream, ping-pong wgrad)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/s13
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s13/pytest_gpu.txt 2>&1; rc=$?; tail -5 gpurun_out/s13/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s13/smoke.txt 2>&1 || exit 1
tail -2 gpurun_out/s13/smoke.txt
timeout -k 10 300 python -u bench.py > gpurun_out/s13/bench_default.json 2> gpurun_out/s13/bench_default.err || exit 1
tail -1 gpurun_out/s13/bench_default.json | cut -c1-220
