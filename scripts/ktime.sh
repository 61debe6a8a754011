#!/usr/bin/env bash
# Per-kernel times of a command under rocprofv3 (kernel trace only): prints "<avg_us> <calls> <name>".
#   bash scripts/ktime.sh TAG ./bench/native/bin/attn_bwd_store 64
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/ktime_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o k -- "$@" > "$out.log" 2>&1
python3 - "$out/k_kernel_stats.csv" "$tag" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{sys.argv[2]:>14s} {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4s}  {r['Name'][:90]}")
PY
