#!/usr/bin/env bash
# Same-box interleaved A/B/C... of bench.py under N environments (2 rounds):
#   bash scripts/abn.sh "ENV_A=1" "ENV_B=1" "ENV_C=1 ENV_D=2" -- [bench args...]
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
envs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
[ $# -gt 0 ] && shift
for round in 1 2; do
  for e in "${envs[@]}"; do
    v=$(env $e timeout -k 10 300 python bench.py "$@" 2>/dev/null | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
    echo "[$e] round$round: $v tok/s"
  done
done
