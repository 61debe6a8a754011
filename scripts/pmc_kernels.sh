#!/usr/bin/env bash
# Two hardware-counter passes (one rocprofv3 run per counter set, kernel trace only) over a
# command; prints per-kernel averages per dispatch and the derived MFMA-busy / wait shares.
#   OUT=gpurun_out/pmc TAG=fc bash scripts/pmc_kernels.sh python3 bench/micro.py fgemm1 768 3072 0 0 131072
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}; TAG=${TAG:-run}
mkdir -p "$OUT"
sets=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
      "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAVES")
i=0
for set in "${sets[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$OUT/$TAG$i" -o pmc -- "$@" \
    > "$OUT/$TAG$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -5 "$OUT/$TAG$i.log"; exit 1; }
done
python3 - "$OUT" "$TAG" <<'PY' | tee "$OUT/$TAG.summary.txt"
import collections, csv, glob, sys
out, tag = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(collections.Counter)
for f in glob.glob(f"{out}/{tag}[0-9]/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"][:80]
        agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[n][r["Counter_Name"]] += 1
for n, c in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CYCLES", 0)):
    avg = {k: v / max(1, cnt[n][k]) for k, v in c.items()}
    wc = avg.get("SQ_WAVE_CYCLES", 0) or 1
    busy = avg.get("SQ_BUSY_CYCLES", 0) or 1
    print(n)
    print("   " + "  ".join(f"{k}={v:.4g}" for k, v in sorted(avg.items())))
    # SQ_VALU_MFMA_BUSY_CYCLES counts cycles (summed over SIMDs); SQ_BUSY_CYCLES counts per SE quad-cycles
    print(f"   wait_any {avg.get('SQ_WAIT_ANY', 0) / wc:.3f}  wait_inst {avg.get('SQ_WAIT_INST_ANY', 0) / wc:.3f}"
          f"  active {avg.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f}  (shares of wave cycles)"
          f"  lds_conflict/idx {avg.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, avg.get('SQ_LDS_IDX_ACTIVE', 0)):.3f}")
PY
