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
# newest one (data order replayed per rank, see training/trainer.py).  The newest checkpoint and
# the restart's run-id suffix come from `python -m llmtrain.launch` (unit-tested); the suffix is
# the Job's UID (JOB_UID, from the pods' controller-uid label), so all ranks of one restarted gang
# write into the same run directory.
#
# LAUNCH_MODE=torchrun (k8s/job-1pod8gpu.yaml): ONE pod owns all NPROC GPUs of the node and
# torchrun starts one rank per GPU inside it — the fallback when the device plugin cannot give
# one-GPU pods access to their peers' render nodes (RCCL would leave xGMI P2P).
set -euo pipefail

: "${LAUNCH_MODE:=pod-per-gpu}"
: "${MASTER_PORT:=29500}"
: "${JOB_NAME:?JOB_NAME must be set}"
: "${CONFIG_PATH:=/config/train.yaml}"
: "${RUNS_ROOT:=/app/runs}"
: "${RUN_ID:=${JOB_NAME}}"
export HSA_ENABLE_IPC_MODE_LEGACY=0

if [ "$LAUNCH_MODE" = torchrun ]; then
  : "${NPROC:=8}"
  RANK=0
else
  : "${JOB_COMPLETION_INDEX:?JOB_COMPLETION_INDEX is not set (not an IndexedJob?)}"
  : "${WORLD_SIZE:?WORLD_SIZE must be set}"
  export RANK="$JOB_COMPLETION_INDEX"
  export LOCAL_RANK=0
fi

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

if [ "$LAUNCH_MODE" = torchrun ]; then
  MASTER_ADDR=127.0.0.1
else
  MASTER_ADDR=$(resolve_master) || { echo "ERROR: could not resolve rank-0 address" >&2; exit 1; }
fi
export MASTER_ADDR
log "mode=${LAUNCH_MODE} WORLD_SIZE=${WORLD_SIZE:-$NPROC} MASTER_ADDR=${MASTER_ADDR}:${MASTER_PORT} visible GPUs: $(python -c 'import torch;print(torch.cuda.device_count())')"

# newest checkpoint of this job across its run directories (the original and any restarts)
LATEST=$(python -m llmtrain.launch latest-checkpoint --runs-root "$RUNS_ROOT" --run-id "$RUN_ID" || true)
RESUME=()
RUN_ARGS=(--run-id "$RUN_ID")
if [ -n "$LATEST" ]; then
  RESUME=(--resume "$LATEST")
  # a restarted job writes into a fresh run directory next to the original one, named by the
  # Job incarnation's UID so every rank of the gang picks the same one
  TAG=$(python -m llmtrain.launch restart-tag) || { echo "ERROR: JOB_UID not set" >&2; exit 1; }
  RUN_ARGS=(--run-id "${RUN_ID}-restart-${TAG}")
  log "resuming from ${LATEST}"
fi

if [ "$LAUNCH_MODE" = torchrun ]; then
  log "exec torchrun --nproc-per-node ${NPROC} -m llmtrain train --config ${CONFIG_PATH} ${RUN_ARGS[*]} ${RESUME[*]:-}"
  exec python -m torch.distributed.run --nnodes 1 --nproc-per-node "$NPROC" --master-addr 127.0.0.1 \
    --master-port "$MASTER_PORT" -m llmtrain train --config "$CONFIG_PATH" "${RUN_ARGS[@]}" "${RESUME[@]}"
fi
log "exec python -m llmtrain train --config ${CONFIG_PATH} ${RUN_ARGS[*]} ${RESUME[*]:-}"
exec python -m llmtrain train --config "$CONFIG_PATH" "${RUN_ARGS[@]}" "${RESUME[@]}"
