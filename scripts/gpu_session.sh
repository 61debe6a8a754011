#!/usr/bin/env bash
# One GPU-box session, as a list of named steps (each with its own time limit; the session stops
# at the first failing step and never retries a GPU step):
#
#   bash scripts/gpu_session.sh [-o OUTDIR] STEP [STEP ...]
#
#   tests[:EXPR]       pytest -m gpu (one process, per-test timeout; EXPR: pytest -k expression)
#   smoke              __graft_entry__.smoke()
#   bench[:MB[:ARGS]]  bench.py --gpus 1 at micro-batch MB (default 128); ARGS: extra flags, ',' for ' '
#   prof[:MB[:ARGS]]   rocprofv3 kernel trace of a short bench run -> OUT/kernel_stats_TAG.txt (per step;
#                      TAG = $PROF_TAG or mbMB; ARGS: extra bench flags, ',' for ' ')
#   tune[:MB[:ARGS]]   scripts/tune_gemms.sh (TunableOp pass over the bench's library GEMMs, AB=0)
#   det[:ENV]          bench/determinism_probe.py (ENV e.g. LLMTRAIN_WGRAD_STREAM=0)
#   detruns[:ENV]      3 whole deterministic runs of DET_STEPS (400) steps, compared step by step
#   gloo2              bench.py --gpus 2 --backend gloo on the one GPU (rehearses the 2-rank path)
#   micro:WHAT[:ARGS]  bench/micro.py WHAT ARGS
#   parity[:ARGS]      bench/parity.py ARGS
#   repeat[:M]         bench/repeat_check.py M
#   ab:ENVA|ENVB[:ARGS] same-box interleaved bench.py A/B (scripts/abn.sh)
#   wpp:ARGS           bench/wgrad_pp.py ARGS (weight-gradient GEMM numerics / timing)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/session
if [ "${1:-}" = "-o" ]; then OUT=$2; shift 2; fi
mkdir -p "$OUT"

run() {  # run NAME LIMIT CMD... : stdout/stderr to OUT/NAME.log (NAME_2, _3.. when repeated), tail shown, exit on failure
  local name=$1 limit=$2; shift 2
  local n=2 base=$name
  while [ -e "$OUT/$name.log" ]; do name=${base}_$n; n=$((n + 1)); done
  echo "== $name: $*"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n "${TAIL:-3}" "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; exit $rc; fi
}

for step in "$@"; do
  kind=${step%%:*}; arg=""; [ "$kind" != "$step" ] && arg=${step#*:}
  case $kind in
    tests) if [ -n "$arg" ]; then
        run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$arg"
      else
        run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
      fi ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)
      mb=${arg%%:*}; mb=${mb:-128}; extra=""; [[ "$arg" == *:* ]] && extra=${arg#*:}
      run "bench_mb$mb" 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --micro-batch "$mb" ${extra//,/ } ;;
    prof)
      mb=${arg%%:*}; mb=${mb:-128}; extra=""; [[ "$arg" == *:* ]] && extra=${arg#*:}
      tag=${PROF_TAG:-mb$mb}; d="$OUT/prof_$tag"; mkdir -p "$d"
      run "prof_$tag" 600 rocprofv3 --kernel-trace --output-format rocpd -d "$d" -o run -- \
        python3 bench.py --gpus 1 --steps 6 --warmup 3 --micro-batch "$mb" ${extra//,/ }
      db=$(find "$d" -name "*.db" | head -1)
      python3 scripts/rocpd_stats.py "$db" 3 40 > "$OUT/kernel_stats_$tag.txt" 2>&1 || true
      python3 scripts/rocpd_timeline.py "$db" 3 > "$OUT/timeline_$tag.txt" 2>&1 || true
      rm -f "$db"
      cat "$OUT/kernel_stats_$tag.txt" ;;
    det)
      name=det${arg:+_${arg//[^A-Za-z0-9]/_}}
      echo "== $name"
      env ${arg} timeout -k 10 300 python -u bench/determinism_probe.py --steps 150 --reps 3 > "$OUT/$name.jsonl" 2> "$OUT/$name.err"
      rc=$?; tail -n 2 "$OUT/$name.jsonl"; [ $rc -le 1 ] || { echo "== $name FAILED rc=$rc"; tail -20 "$OUT/$name.err"; exit $rc; } ;;
    detruns)
      name=detruns${arg:+_${arg//[^A-Za-z0-9]/_}}
      echo "== $name"
      env ${arg} timeout -k 10 400 python -u bench/determinism_probe.py --runs 3 --steps ${DET_STEPS:-400} > "$OUT/$name.jsonl" 2> "$OUT/$name.err"
      rc=$?; tail -n 4 "$OUT/$name.jsonl"; [ $rc -le 1 ] || { echo "== $name FAILED rc=$rc"; tail -20 "$OUT/$name.err"; exit $rc; } ;;
    gloo2) run gloo2 400 python -u bench.py --gpus 2 --backend gloo --steps 4 --warmup 2 --micro-batch 16 ;;
    micro) what=${arg%%:*}; rest=""; [[ "$arg" == *:* ]] && rest=${arg#*:}
      run "micro_${what}" 400 python -u bench/micro.py "$what" ${rest//,/ } ;;
    parity) run parity 1100 python -u bench/parity.py ${arg//,/ } ;;
    repeat) run repeat 400 python -u bench/repeat_check.py ${arg:-32768} ;;
    ab) envs=${arg%%:*}; rest=""; [[ "$arg" == *:* ]] && rest=${arg#*:}
      IFS='|' read -r -a E <<< "$envs"
      run ab 1000 bash scripts/abn.sh "${E[@]}" -- ${rest//,/ } ;;
    tune)
      mb=${arg%%:*}; mb=${mb:-128}; extra=""; [[ "$arg" == *:* ]] && extra=${arg#*:}
      run "tune_$mb" 1000 env MB="$mb" BENCH_ARGS="${extra//,/ }" AB=0 bash scripts/tune_gemms.sh ;;
    wpp) run "wpp_${arg%%,*}" 300 python -u bench/wgrad_pp.py ${arg//,/ } ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== session done"
