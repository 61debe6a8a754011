#!/usr/bin/env bash
# End-to-end check of the 8-pod IndexedJob on a cluster with an 8x MI355X node
# (label it: kubectl label node <node> llmtrain.amd.com/mi355x-node=true).
#   k8s/test_e2e.sh [--no-cleanup] [--image llmtrain-mi355x:dev] [--timeout 1800]
# Asserts: the Job completes, every pod exits 0, rank 0 logged "final_step=" / the step lines and
# nothing else printed a summary, the run directory on the runs PVC has checkpoints, logs,
# config.yaml and meta.json, and (if enabled) the MLflow SQLite store is non-empty.
set -euo pipefail
CLEANUP=1
IMAGE=llmtrain-mi355x:dev
TIMEOUT=1800
while [ $# -gt 0 ]; do
  case "$1" in
    --no-cleanup) CLEANUP=0 ;;
    --image) IMAGE="$2"; shift ;;
    --timeout) TIMEOUT="$2"; shift ;;
    *) echo "unknown arg $1" >&2; exit 2 ;;
  esac
  shift
done
here="$(cd "$(dirname "$0")" && pwd)"
manifests=("$here/rbac.yaml" "$here/storage.yaml" "$here/configmap.yaml" "$here/service.yaml" "$here/job.yaml")
cleanup() { [ "$CLEANUP" = 1 ] && kubectl delete -f "$here/job.yaml" --ignore-not-found >/dev/null 2>&1 || true; }
trap cleanup EXIT

kubectl apply "${manifests[@]/#/-f}"
kubectl set image job/llmtrain trainer="$IMAGE" >/dev/null 2>&1 || true
echo "waiting up to ${TIMEOUT}s for job/llmtrain ..."
kubectl wait --for=condition=complete --timeout="${TIMEOUT}s" job/llmtrain

fail=0
for pod in $(kubectl get pods -l app=llmtrain -o jsonpath='{.items[*].metadata.name}'); do
  code=$(kubectl get pod "$pod" -o jsonpath='{.status.containerStatuses[0].state.terminated.exitCode}')
  [ "$code" = "0" ] || { echo "FAIL: $pod exited $code"; fail=1; }
done
rank0=$(kubectl get pods -l app=llmtrain,batch.kubernetes.io/job-completion-index=0 -o jsonpath='{.items[0].metadata.name}')
logs=$(kubectl logs "$rank0")
grep -q "final_step=" <<<"$logs" || { echo "FAIL: rank 0 printed no summary"; fail=1; }
grep -q "step=" <<<"$logs" || { echo "FAIL: no step log lines"; fail=1; }
grep -q "entrypoint\[rank 0\]: exec python" <<<"$logs" || { echo "FAIL: entrypoint did not exec"; fail=1; }

# inspect the runs PVC through a throwaway pod
kubectl run llmtrain-inspect --rm -i --restart=Never --image=busybox \
  --overrides='{"spec":{"volumes":[{"name":"runs","persistentVolumeClaim":{"claimName":"runs-pvc"}},{"name":"mlflow","persistentVolumeClaim":{"claimName":"mlflow-pvc"}}],"containers":[{"name":"c","image":"busybox","command":["sh","-c","ls /runs/*/checkpoints/step_*.pt && ls /runs/*/logs/train.log /runs/*/config.yaml /runs/*/meta.json && test -s /mlflow/mlflow.db"],"volumeMounts":[{"name":"runs","mountPath":"/runs"},{"name":"mlflow","mountPath":"/mlflow"}]}]}}' \
  || { echo "FAIL: run directory / mlflow artifacts missing"; fail=1; }

[ "$fail" = 0 ] && echo "E2E OK" || { echo "E2E FAILED"; exit 1; }
