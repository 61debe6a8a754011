# weight-gradient ping-pong kernel: fill-op placement variants (LLMT_WPP_PLACE), op level
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/s4
for rnd in 1 2; do
for pl in 0 1 2; do
  for m in 131072 32768; do
    LLMT_WPP_PLACE=$pl timeout -k 10 120 python -u bench/wgrad_pp.py time --tokens $m --only pp_auto,pp_slab_bias > gpurun_out/s4/place${pl}_m${m}_r$rnd.log 2>&1 || exit 1
  done
done
done
LLMT_WPP_PLACE=1 timeout -k 10 120 python -u bench/wgrad_pp.py check > gpurun_out/s4/check_place1.log 2>&1; tail -1 gpurun_out/s4/check_place1.log
LLMT_WPP_PLACE=2 timeout -k 10 120 python -u bench/wgrad_pp.py check > gpurun_out/s4/check_place2.log 2>&1; tail -1 gpurun_out/s4/check_place2.log
for f in gpurun_out/s4/place*.log; do echo "$f"; grep -v amdgpu "$f" | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('  ', d['gemm'], d['variant'], d['ms'], d['TFLOPs'])"; done
