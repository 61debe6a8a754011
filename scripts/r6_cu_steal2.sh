#!/usr/bin/env bash
# Round 6: which kernels slow down beside a resident thief kernel (bench/cu_steal.py)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6_cu_steal2}
mkdir -p "$OUT"
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; tail -n 6 "$OUT/$name.log"; [ $rc -eq 0 ] || { echo "== $name FAILED rc=$rc"; exit $rc; }; }
step k1 200 python -u bench/cu_steal.py --blocks 0 1 3 8 --rounds 1
step prof_free 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_free" -o run -- python3 -u bench/cu_steal.py --blocks 0 --rounds 1 --thief-ms 2000 --steps 5
step prof_thief 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_thief" -o run -- python3 -u bench/cu_steal.py --blocks 8 --rounds 1 --thief-ms 2000 --steps 5
echo done
