#!/usr/bin/env bash
# Round 6: weight-gradient L2 prefetch distance A/B (release = off)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6_wpf}
mkdir -p "$OUT"
ext() { [ "$1" = rel ] && echo "" || echo "llmtrain/ops/variants/_llmtrain_hip_$1.so"; }
LLMTRAIN_HIP_EXT=$(ext pf6) timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k wgrad > "$OUT/tests_pf6.log" 2>&1 || { tail -20 "$OUT/tests_pf6.log"; exit 1; }
echo "tests pf6: $(tail -1 "$OUT/tests_pf6.log")"
for r in 1 2; do
  for v in rel pf4 pf6 pf8; do
    LLMTRAIN_HIP_EXT=$(ext $v) timeout -k 10 200 python -u bench/wgrad_pp.py time --model gpt2-124m --tokens 131072 --only pp_auto 2>/dev/null | grep variant | sed "s/^{/{\"build\": \"$v\", /" >> "$OUT/time_124m.jsonl" || exit 1
    LLMTRAIN_HIP_EXT=$(ext $v) timeout -k 10 200 python -u bench/wgrad_pp.py time --model gpt2-xl --tokens 32768 --only pp_slab 2>/dev/null | grep variant | sed "s/^{/{\"build\": \"$v\", /" >> "$OUT/time_xl.jsonl" || exit 1
  done
done
python3 - "$OUT" <<'PY'
import json, sys, collections
for f in ("time_124m", "time_xl"):
    d = collections.defaultdict(list)
    for l in open(f"{sys.argv[1]}/{f}.jsonl"):
        r = json.loads(l); d[(r["gemm"], r["build"])].append(r["ms"])
    for k in sorted(d): print(f, k, d[k])
PY
echo done
