#!/usr/bin/env bash
# Counter passes over the weight-gradient kernel (one shape), each set in its own rocprofv3 run.
#   SHAPE="2304 768 131072" OUT=gpurun_out/wgpmc bash scripts/wg_pmc.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/wgpmc}
mkdir -p "$OUT"
SHAPE=${SHAPE:-"2304 768 131072"}
timeout -k 10 120 python3 bench/wgrad_one.py $SHAPE 10 > "$OUT/time.log" 2>&1
i=0
for set in "FETCH_SIZE GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$OUT/p$i" -o pmc -- \
    python3 bench/wgrad_one.py $SHAPE 3 > "$OUT/p$i.log" 2>&1
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(float)
cnt = collections.Counter()
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wgrad" not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[r["Counter_Name"]] += 1
for k in sorted(agg):
    print(f"{k:32s} {agg[k] / max(1, cnt[k]):.4g} (per-dispatch avg over {cnt[k]} rows)")
PY
