# weight-gradient ping-pong kernel: 4 vs 5 ring slots (LLMT_WPP_SLOTS), op level, 2 rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/s5
LLMT_WPP_SLOTS=5 timeout -k 10 120 python -u bench/wgrad_pp.py check > gpurun_out/s5/check_slots5.log 2>&1; echo "check5 rc=$?"; tail -1 gpurun_out/s5/check_slots5.log
for rnd in 1 2; do
for sl in 4 5; do
  for m in 131072 32768; do
    LLMT_WPP_SLOTS=$sl timeout -k 10 120 python -u bench/wgrad_pp.py time --tokens $m --only pp_slab,pp_slab_bias > gpurun_out/s5/slots${sl}_m${m}_r$rnd.log 2>&1 || exit 1
  done
done
done
LLMT_WPP_SLOTS=5 timeout -k 10 120 python -u bench/wgrad_pp.py time --model head --only pp_auto > gpurun_out/s5/slots5_head.log 2>&1 || exit 1
LLMT_WPP_SLOTS=4 timeout -k 10 120 python -u bench/wgrad_pp.py time --model head --only pp_auto > gpurun_out/s5/slots4_head.log 2>&1 || exit 1
for f in gpurun_out/s5/slots*.log; do echo "$f"; grep -v amdgpu "$f" | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('  ', d['gemm'], d['variant'], d['ms'], d['TFLOPs'])"; done
