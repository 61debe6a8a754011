#!/usr/bin/env bash
# Repeat bench.py N times under an environment and print value / ms per step (stderr tail on failure).
#   bash scripts/rep.sh N "ENV=1 ENV2=0" [bench args...]
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
n=$1; envs=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 "$n"); do
  if env $envs timeout -k 10 300 python bench.py "$@" > gpurun_out/rep.out 2> gpurun_out/rep.err; then
    python3 -c "import json; d=json.loads(open('gpurun_out/rep.out').read()); print('[$envs] run $i:', d['value'], d['ms_per_step'])"
  else
    echo "[$envs] run $i FAILED rc=$?"; tail -5 gpurun_out/rep.err; exit 1
  fi
done
