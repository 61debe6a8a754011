#!/usr/bin/env bash
# Round 6: step time with k CUs held by a concurrent kernel (bench/cu_steal.py), release build and
# the variant that sizes grids for 16 CUs fewer (LLMT_CU_RESERVE=16)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6_cu_steal}
mkdir -p "$OUT"
V=llmtrain/ops/variants/_llmtrain_hip_cures16.so
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; tail -n 9 "$OUT/$name.log"; [ $rc -eq 0 ] || { echo "== $name FAILED rc=$rc"; exit $rc; }; }
step release 300 python -u bench/cu_steal.py --blocks 0 8 16 32 64
LLMTRAIN_HIP_EXT=$V step reserve16 300 python -u bench/cu_steal.py --blocks 0 16
echo done
