#!/usr/bin/env bash
# IndexedJob bootstrap for one-GPU-per-pod data parallelism on an 8x MI355X node.
#
# Contract with the trainer (same env contract as the reference entrypoint):
#   RANK        = JOB_COMPLETION_INDEX
#   WORLD_SIZE  = from the Job spec
#   LOCAL_RANK  = 0  (each pod is allocated exactly one GPU via amd.com/gpu: 1, so the process
#                     sees it as HIP device 0 — the reference used the index because it ran on CPU)
#   MASTER_ADDR = rank 0's pod, resolved through the headless Service DNS name
#                 <job>-0.<service>; falls back to the Kubernetes API (podIP of index 0) when the
#                 pod has no subdomain
#   MASTER_PORT = from the Job spec
# Automatic recovery: every pod passes --run-id "$RUN_ID"; if the job already wrote checkpoints to
# the shared runs PVC (a replaced pod, or the whole Job restarted) every rank resumes from the
# newest one (data order replayed per rank, see training/trainer.py).
set -euo pipefail

: "${JOB_COMPLETION_INDEX:?JOB_COMPLETION_INDEX is not set (not an IndexedJob?)}"
: "${WORLD_SIZE:?WORLD_SIZE must be set}"
: "${MASTER_PORT:=29500}"
: "${JOB_NAME:?JOB_NAME must be set}"
: "${CONFIG_PATH:=/config/train.yaml}"
: "${RUNS_ROOT:=/app/runs}"
: "${RUN_ID:=${JOB_NAME}}"

export RANK="$JOB_COMPLETION_INDEX"
export LOCAL_RANK=0
export HSA_ENABLE_IPC_MODE_LEGACY=0

log() { echo "entrypoint[rank ${RANK}]: $*"; }

resolve_master() {
  if [ "$RANK" -eq 0 ] && [ -n "${POD_IP:-}" ]; then
    echo "$POD_IP"; return 0
  fi
  if [ -n "${SERVICE_NAME:-}" ]; then
    local host="${JOB_NAME}-0.${SERVICE_NAME}"
    for _ in $(seq 1 60); do
      ip=$(getent hosts "$host" | awk '{print $1}' | head -n1 || true)
      if [ -n "$ip" ]; then echo "$ip"; return 0; fi
      sleep 2
    done
  fi
  # fallback: ask the API server for index 0's pod IP (needs the rbac.yaml role)
  local sa=/var/run/secrets/kubernetes.io/serviceaccount
  local ns; ns=$(cat "$sa/namespace")
  local url="https://kubernetes.default.svc/api/v1/namespaces/${ns}/pods?labelSelector=batch.kubernetes.io/job-completion-index=0,job-name=${JOB_NAME}"
  for _ in $(seq 1 60); do
    ip=$(curl -s --cacert "$sa/ca.crt" -H "Authorization: Bearer $(cat "$sa/token")" "$url" \
         | jq -r '.items[0].status.podIP // empty' || true)
    if [ -n "$ip" ] && [ "$ip" != "null" ]; then echo "$ip"; return 0; fi
    sleep 2
  done
  return 1
}

MASTER_ADDR=$(resolve_master) || { echo "ERROR: could not resolve rank-0 address" >&2; exit 1; }
export MASTER_ADDR
log "WORLD_SIZE=${WORLD_SIZE} MASTER_ADDR=${MASTER_ADDR}:${MASTER_PORT} visible GPUs: $(python -c 'import torch;print(torch.cuda.device_count())')"

# newest checkpoint of this job across its run directories (the original and any restarts)
LATEST=$(ls -1 "${RUNS_ROOT}/${RUN_ID}"*/checkpoints/step_*.pt 2>/dev/null \
         | awk -F'step_' '{print $NF" "$0}' | sort -n | tail -n1 | cut -d' ' -f2- || true)
RESUME=()
RUN_ARGS=(--run-id "$RUN_ID")
if [ -n "$LATEST" ]; then
  RESUME=(--resume "$LATEST")
  # a restarted job writes into a fresh run directory next to the original one
  RUN_ARGS=(--run-id "${RUN_ID}-restart-${RESTART_TAG:-$(date +%Y%m%d%H%M%S)}")
  log "resuming from ${LATEST}"
fi

log "exec python -m llmtrain train --config ${CONFIG_PATH} ${RUN_ARGS[*]} ${RESUME[*]:-}"
exec python -m llmtrain train --config "$CONFIG_PATH" "${RUN_ARGS[@]}" "${RESUME[@]}"
