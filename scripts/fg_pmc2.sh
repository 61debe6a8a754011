#!/usr/bin/env bash
# L2 counters over one fused-GEMM shape (NT and NN): TCC hit/miss/requests.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/fgpmc2}
mkdir -p "$OUT"
i=0
for shape in "768 3072 0 0" "768 3072 0 1"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum --output-format csv -d "$OUT/p$i" -o pmc -- \
    python3 bench/micro.py fgemm1 $shape > "$OUT/p$i.log" 2>&1
  grep TFLOPs "$OUT/p$i.log" || true
  python3 - "$OUT/p$i" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(float); cnt = collections.Counter()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gemm_fused" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
for k in sorted(agg):
    print(f"  {k:24s} {agg[k] / max(1, cnt[k]):.4g}")
PY
done
