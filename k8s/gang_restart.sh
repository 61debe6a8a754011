#!/usr/bin/env bash
# Gang-restart controller for the training IndexedJob.
#
#   k8s/gang_restart.sh [--job k8s/job.yaml] [--name llmtrain] [--max-restarts 3] [--timeout 3600]
#                       [--poll 5]
#
# The Job's podFailurePolicy fails the WHOLE Job as soon as any rank fails (a replaced pod cannot
# rejoin a live RCCL group; its peers would otherwise block in a collective until the watchdog
# fires).  This controller turns that fast failure into a fast recovery: it (re)creates the Job,
# waits for Complete or Failed, and on Failed deletes it (all pods) and creates it again, up to
# --max-restarts times.  Every rank of the new incarnation finds the newest checkpoint on the runs
# PVC and resumes from it (k8s/entrypoint.sh), so a restart costs the steps since the last
# checkpoint plus pod start-up, not a 900 s collective timeout.
#
# Exit status: 0 = the Job completed; 1 = it failed more than --max-restarts times or timed out.
# Prints one "gang_restart: ..." line per event (attempts, terminal states, failed pods).
set -euo pipefail

JOB_MANIFEST="$(cd "$(dirname "$0")" && pwd)/job.yaml"
NAME=llmtrain
MAX_RESTARTS=3
TIMEOUT=3600
POLL=5
KUBECTL=${KUBECTL:-kubectl}
while [ $# -gt 0 ]; do
  case "$1" in
    --job) JOB_MANIFEST="$2"; shift ;;
    --name) NAME="$2"; shift ;;
    --max-restarts) MAX_RESTARTS="$2"; shift ;;
    --timeout) TIMEOUT="$2"; shift ;;
    --poll) POLL="$2"; shift ;;
    -h|--help) sed -n '2,18p' "$0"; exit 0 ;;
    *) echo "gang_restart: unknown argument $1" >&2; exit 2 ;;
  esac
  shift
done

log() { echo "gang_restart: $*"; }

job_state() {
  # Complete | Failed | Running (no terminal condition yet)
  local conds
  conds=$($KUBECTL get job "$NAME" -o jsonpath='{range .status.conditions[?(@.status=="True")]}{.type}{" "}{end}' 2>/dev/null || true)
  case " $conds " in
    *" Complete "*) echo Complete ;;
    *" Failed "*) echo Failed ;;
    *) echo Running ;;
  esac
}

report_failures() {
  $KUBECTL get pods -l "job-name=$NAME" \
    -o jsonpath='{range .items[*]}{.metadata.name}{" "}{.status.containerStatuses[0].state.terminated.exitCode}{" "}{.status.containerStatuses[0].state.terminated.reason}{"\n"}{end}' \
    2>/dev/null | while read -r pod code reason; do
      [ -n "$pod" ] && [ "${code:-0}" != "0" ] && log "  failed pod $pod exit=${code:-?} reason=${reason:-?}"
    done || true
}

deadline=$(( $(date +%s) + TIMEOUT ))
attempt=0
while :; do
  $KUBECTL delete job "$NAME" --ignore-not-found --cascade=foreground --wait=true >/dev/null
  log "attempt $attempt: creating job/$NAME from $JOB_MANIFEST"
  $KUBECTL apply -f "$JOB_MANIFEST" >/dev/null
  state=Running
  while [ "$state" = Running ]; do
    if [ "$(date +%s)" -ge "$deadline" ]; then
      log "timed out after ${TIMEOUT}s (attempt $attempt still running)"
      exit 1
    fi
    sleep "$POLL"
    state=$(job_state)
  done
  if [ "$state" = Complete ]; then
    log "job/$NAME complete after $attempt restart(s)"
    exit 0
  fi
  log "attempt $attempt: job/$NAME failed"
  report_failures
  attempt=$(( attempt + 1 ))
  if [ "$attempt" -gt "$MAX_RESTARTS" ]; then
    log "giving up after $MAX_RESTARTS restart(s)"
    exit 1
  fi
  log "restarting the whole gang; ranks resume from the newest checkpoint"
done
