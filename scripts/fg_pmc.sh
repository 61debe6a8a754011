#!/usr/bin/env bash
# Counter passes over the fused GEMM (one shape): PMC sets each in their own rocprofv3 run.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/fgpmc}
mkdir -p "$OUT"
SHAPE=${SHAPE:-"768 3072 0 0"}
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$OUT/p$i" -o pmc -- \
    python3 bench/micro.py fgemm1 $SHAPE > "$OUT/p$i.log" 2>&1
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gemm_fused" not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]]["v"] += float(r["Counter_Value"])
        cnt[r["Counter_Name"]] += 1
for k in sorted(agg):
    print(f"{k:32s} {agg[k]['v'] / max(1, cnt[k]):.4g} (per-dispatch avg over {cnt[k]} rows)")
PY
