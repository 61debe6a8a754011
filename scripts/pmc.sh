#!/usr/bin/env bash
# Hardware-counter pass (kernel-trace only, no sys/runtime trace: see gpurun rules) over a command.
#   PMC="SQ_WAVES SQ_INSTS_VALU ..." OUT=gpurun_out/pmc bash scripts/pmc.sh python3 bench/micro.py attn
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}
mkdir -p "$OUT"
timeout -k 10 600 rocprofv3 --kernel-trace --pmc ${PMC} --output-format csv -d "$OUT" -o pmc -- "$@" > "$OUT/run.log" 2>&1
