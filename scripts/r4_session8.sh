# register-staged fill (2 slots): which part of the fill costs — skeletons 1 (none), 2 (loads only), 3 (LDS writes only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/s8
for rnd in 1 2; do
for sk in 0 1 2 3; do
  LLMT_WPP_FILL=1 LLMT_WPP_SLOTS=2 LLMT_WPP_SKEL=$sk timeout -k 10 120 python -u bench/wgrad_pp.py time --tokens 131072 --only pp_slab > gpurun_out/s8/skel${sk}_r$rnd.log 2>&1 || exit 1
done
done
for f in gpurun_out/s8/skel*.log; do echo "$f"; grep -v amdgpu "$f" | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('  ', d['gemm'], d['variant'], d['ms'], d['TFLOPs'])"; done
