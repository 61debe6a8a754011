#!/usr/bin/env bash
# Same-box interleaved A/B/C/... of bench.py over N environments, ROUNDS rounds (default 2):
#   bash scripts/abn.sh "X=0" "LLMTRAIN_FGEMM_ANY_SIZE=dx_gelu" ... [-- bench args]
# Each line: <env> round<r>: <tok/s>.  Logs under gpurun_out/abn/.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abn
envs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
for round in $(seq 1 "${ROUNDS:-2}"); do
  for i in "${!envs[@]}"; do
    log="gpurun_out/abn/cfg${i}_r${round}.log"
    env ${envs[$i]} timeout -k 10 300 python bench.py "$@" > "$log" 2>&1 || { echo "bench failed: ${envs[$i]}"; tail -20 "$log"; exit 1; }
    echo "${envs[$i]} round$round: $(tail -1 "$log" | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
done
