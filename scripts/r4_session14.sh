# ping-pong weight-gradient kernel: memory-side counters (HBM fetch, L2 hits) on qkv at M = 131072
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/s14
run() {  # run TAG COUNTERS...
  local tag=$1; shift
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d gpurun_out/s14/$tag -o pmc -- \
    python3 bench/wgrad_pp.py one --gemm qkv --variant pp --reps 5 > gpurun_out/s14/$tag.log 2>&1 || { echo "pass $tag failed"; tail -3 gpurun_out/s14/$tag.log; exit 1; }
}
run a FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE
run b TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum
run c WRITE_SIZE TCC_EA0_WRREQ_sum
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/s14/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wgrad_pp_kernel" in r["Kernel_Name"]:
            agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c} mean {sum(v)/len(v):.4g} over {len(v)} dispatches")
PY
