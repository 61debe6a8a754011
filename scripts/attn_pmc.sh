#!/usr/bin/env bash
# Counter passes over the stand-alone attention timers (bench/native/bin, scripts/build_timers.sh),
# one rocprofv3 run per counter set; prints per-kernel averages.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/attnpmc}
B=${B:-32}
mkdir -p "$OUT"
sets=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE"
      "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC SQ_WAVES")
for bin in fwd_new bwd_new; do
  i=0
  for set in "${sets[@]}"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$OUT/$bin$i" -o pmc -- \
      bench/native/bin/$bin "$B" > "$OUT/$bin$i.log" 2>&1
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.defaultdict(collections.Counter)
for f in glob.glob(sys.argv[1] + "/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        k = ("fwd" if "attn_fwd" in n else "bwd" if "attn_bwd_kernel" in n else "delta" if "attn_delta" in n
             else "dq_reduce" if "dq_reduce" in n else None)
        if k:
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[k][r["Counter_Name"]] += 1
for k in agg:
    a = {c: agg[k][c] / max(1, cnt[k][c]) for c in agg[k]}
    print(k)
    for c in sorted(a):
        print(f"  {c:28s} {a[c]:.4g}")
    if a.get("SQ_LDS_IDX_ACTIVE"):
        print(f"  -> LDS bank-conflict cycles / LDS active cycles = {a.get('SQ_LDS_BANK_CONFLICT', 0) / a['SQ_LDS_IDX_ACTIVE']:.3f}")
    if a.get("SQ_INSTS_MFMA"):
        print(f"  -> VALU instructions per MFMA = {a.get('SQ_INSTS_VALU', 0) / a['SQ_INSTS_MFMA']:.1f}")
PY
