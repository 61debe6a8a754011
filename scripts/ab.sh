#!/usr/bin/env bash
# Same-box A/B of bench.py under two environments, alternating A B A B (MI355X boards differ by
# several % in wall time, so only same-box, interleaved comparisons mean anything).
#   bash scripts/ab.sh "ENV_A=1" "ENV_B=1" [bench args...]
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
a=$1; b=$2; shift 2
for round in 1 2; do
  for tag in A B; do
    envs=$([ "$tag" = A ] && echo "$a" || echo "$b")
    v=$(env $envs timeout -k 10 300 python bench.py "$@" 2>/dev/null | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
    echo "$tag[$envs] round$round: $v tok/s"
  done
done
