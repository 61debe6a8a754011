#!/usr/bin/env bash
# End-to-end test of the training IndexedJob (reference k8s/test_e2e.sh: cluster, image, manifests,
# wait, assertions, cleanup), driven through the gang-restart controller.
#
#   k8s/test_e2e.sh --cpu [--inject-failure [STEP]] [--no-cleanup] [--keep-cluster] [--timeout S]
#       kind mode: creates (or reuses) the kind cluster "llmtrain", builds the image and loads it
#       into kind, runs the 2-pod gloo Job (k8s/kind/job-cpu.yaml) on hostPath PVCs, and checks the
#       artifacts straight from the host directories ./runs and ./mlflow-k8s.
#   k8s/test_e2e.sh [--inject-failure [STEP]] [--image IMG] [--no-cleanup] [--timeout S]
#       MI355X mode: an existing cluster with a labelled 8x MI355X node
#       (kubectl label node <node> llmtrain.amd.com/mi355x-node=true), the 8-pod RCCL Job.
#
# --inject-failure STEP sets trainer.extra.fail_at_step=STEP and fail_rank=1 in the Job's config:
# rank 1 crashes once, the podFailurePolicy fails the whole Job immediately, gang_restart.sh
# re-creates it, every rank resumes from the newest checkpoint, and the test asserts the resumed
# run completes (two attempts, a "resuming from" line, the final checkpoint in the restart's run
# directory).
#
# Asserts: the Job completes; every pod of the final attempt exits 0; rank 0 logged the step lines,
# "final_step=" and "entrypoint[rank 0]: exec python"; the run directory holds checkpoints,
# logs/train.log, config.yaml and meta.json; the MLflow SQLite store is non-empty.
set -euo pipefail

MODE=gpu
CLEANUP=1
KEEP_CLUSTER=0
INJECT=""
IMAGE=llmtrain-mi355x:dev
TIMEOUT=1800
CLUSTER=llmtrain
while [ $# -gt 0 ]; do
  case "$1" in
    --cpu) MODE=cpu ;;
    --no-cleanup) CLEANUP=0 ;;
    --keep-cluster) KEEP_CLUSTER=1 ;;
    --inject-failure)
      INJECT=auto
      if [ $# -gt 1 ] && [[ "$2" =~ ^[0-9]+$ ]]; then INJECT="$2"; shift; fi ;;
    --image) IMAGE="$2"; shift ;;
    --timeout) TIMEOUT="$2"; shift ;;
    --cluster-name) CLUSTER="$2"; shift ;;
    -h|--help) sed -n '2,24p' "$0"; exit 0 ;;
    *) echo "unknown arg $1" >&2; exit 2 ;;
  esac
  shift
done

here="$(cd "$(dirname "$0")" && pwd)"
repo="$(cd "$here/.." && pwd)"
work="$(mktemp -d)"
created_cluster=0
log() { echo "e2e: $*"; }
fail=0
check() { if eval "$2"; then log "ok   $1"; else log "FAIL $1"; fail=1; fi; }

need() { command -v "$1" >/dev/null || { echo "e2e: '$1' is required" >&2; exit 2; }; }
need kubectl
need python3

if [ "$MODE" = cpu ]; then
  need kind
  need docker
  JOB="$here/kind/job-cpu.yaml"
  CONFIGMAP="$here/kind/configmap-cpu.yaml"
  STORAGE="$here/kind/storage-kind.yaml"
  [ "$INJECT" = auto ] && INJECT=30  # after the step-20 checkpoint of the 40-step CPU run
else
  JOB="$here/job.yaml"
  CONFIGMAP="$here/configmap.yaml"
  STORAGE="$here/storage.yaml"
  [ "$INJECT" = auto ] && INJECT=75  # after the step-50 checkpoint
fi

cleanup() {
  if [ "$CLEANUP" = 1 ]; then
    kubectl delete job llmtrain --ignore-not-found --wait=false >/dev/null 2>&1 || true
    if [ "$MODE" = cpu ] && [ "$created_cluster" = 1 ] && [ "$KEEP_CLUSTER" = 0 ]; then
      kind delete cluster --name "$CLUSTER" >/dev/null 2>&1 || true
    fi
  fi
  rm -rf "$work"
}
trap cleanup EXIT

# ---- cluster + image (kind mode) --------------------------------------------------------------
if [ "$MODE" = cpu ]; then
  cd "$repo"
  mkdir -p runs mlflow-k8s
  if kind get clusters 2>/dev/null | grep -qx "$CLUSTER"; then
    log "reusing kind cluster $CLUSTER"
  else
    log "creating kind cluster $CLUSTER"
    kind create cluster --name "$CLUSTER" --config "$here/kind/kind-config.yaml"
    created_cluster=1
  fi
  kubectl config use-context "kind-$CLUSTER" >/dev/null
  log "building $IMAGE"
  docker build -q -t "$IMAGE" -f "$here/Dockerfile" "$repo" >/dev/null
  kind load docker-image "$IMAGE" --name "$CLUSTER"
  rm -rf "$repo"/runs/llmtrain* "$repo"/mlflow-k8s/mlflow.db
fi

# ---- manifests (+ optional fault injection in the embedded training config) ------------------
cm="$work/configmap.yaml"
python3 - "$CONFIGMAP" "$cm" "${INJECT:-}" <<'PY'
import sys, yaml
src, dst, inject = sys.argv[1], sys.argv[2], sys.argv[3]
doc = yaml.safe_load(open(src))
if inject:
    cfg = yaml.safe_load(doc["data"]["train.yaml"])
    extra = cfg["trainer"].setdefault("extra", {})
    extra.update(fail_at_step=int(inject), fail_rank=1)
    doc["data"]["train.yaml"] = yaml.safe_dump(cfg, sort_keys=False)
yaml.safe_dump(doc, open(dst, "w"), sort_keys=False)
PY
sed "s#image: llmtrain-mi355x:dev#image: ${IMAGE}#" "$JOB" > "$work/job.yaml"
kubectl apply -f "$here/rbac.yaml" -f "$STORAGE" -f "$cm" -f "$here/service.yaml" >/dev/null
[ -n "$INJECT" ] && log "fault injection: rank 1 crashes at step $INJECT"

# ---- run through the gang-restart controller ------------------------------------------------
ctl_log="$work/gang_restart.log"
set +e
bash "$here/gang_restart.sh" --job "$work/job.yaml" --max-restarts 2 --timeout "$TIMEOUT" | tee "$ctl_log"
ctl_rc=${PIPESTATUS[0]}
set -e
check "job completed (gang_restart exit 0)" "[ $ctl_rc = 0 ]"

for pod in $(kubectl get pods -l app=llmtrain -o jsonpath='{.items[*].metadata.name}'); do
  code=$(kubectl get pod "$pod" -o jsonpath='{.status.containerStatuses[0].state.terminated.exitCode}')
  check "pod $pod exited 0" "[ '$code' = 0 ]"
done
rank0=$(kubectl get pods -l app=llmtrain,batch.kubernetes.io/job-completion-index=0 -o jsonpath='{.items[0].metadata.name}')
kubectl logs "$rank0" > "$work/rank0.log" 2>&1 || true
check "rank 0 logged step lines" "grep -q 'step=' '$work/rank0.log'"
check "rank 0 printed the run summary" "grep -q 'final_step' '$work/rank0.log'"
check "entrypoint exec'd the trainer" "grep -q 'entrypoint\[rank 0\]: exec python' '$work/rank0.log'"
if [ -n "$INJECT" ]; then
  check "first attempt failed fast (FailJob)" "grep -q 'attempt 0: job/llmtrain failed' '$ctl_log'"
  check "second attempt completed" "grep -q 'complete after 1 restart' '$ctl_log'"
  check "ranks resumed from a checkpoint" "grep -q 'resuming from' '$work/rank0.log'"
fi

# ---- artifacts ------------------------------------------------------------------------------
if [ "$MODE" = cpu ]; then
  runs="$repo/runs"
  check "checkpoints on the runs volume" "ls $runs/llmtrain*/checkpoints/step_*.pt >/dev/null 2>&1"
  check "train.log, config.yaml, meta.json" \
    "ls $runs/llmtrain*/logs/train.log $runs/llmtrain*/config.yaml $runs/llmtrain*/meta.json >/dev/null 2>&1"
  check "MLflow store non-empty" "test -s '$repo/mlflow-k8s/mlflow.db'"
  if [ -n "$INJECT" ]; then
    check "restart run reached the final checkpoint" "ls $runs/llmtrain-restart-*/checkpoints/step_000040.pt >/dev/null 2>&1"
  fi
else
  probe='ls /runs/*/checkpoints/step_*.pt && ls /runs/*/logs/train.log /runs/*/config.yaml /runs/*/meta.json && test -s /mlflow/mlflow.db'
  [ -n "$INJECT" ] && probe="$probe && ls -d /runs/llmtrain-restart-*"
  overrides=$(python3 - "$probe" <<'PY'
import json, sys
print(json.dumps({"spec": {
    "volumes": [{"name": "runs", "persistentVolumeClaim": {"claimName": "runs-pvc"}},
                {"name": "mlflow", "persistentVolumeClaim": {"claimName": "mlflow-pvc"}}],
    "containers": [{"name": "c", "image": "busybox", "command": ["sh", "-c", sys.argv[1]],
                    "volumeMounts": [{"name": "runs", "mountPath": "/runs"},
                                     {"name": "mlflow", "mountPath": "/mlflow"}]}]}}))
PY
)
  check "run directory + MLflow artifacts on the PVCs" \
    "kubectl run llmtrain-inspect --rm -i --restart=Never --image=busybox --overrides='$overrides' >/dev/null"
fi

if [ "$fail" = 0 ]; then echo "E2E OK"; else echo "E2E FAILED"; exit 1; fi
