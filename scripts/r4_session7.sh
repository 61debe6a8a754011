# weight-gradient ping-pong kernel: LDS-DMA fills vs register-staged fills (LLMT_WPP_FILL=1, 4 / 2 slots)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/s7
LLMT_WPP_FILL=1 timeout -k 10 120 python -u bench/wgrad_pp.py check > gpurun_out/s7/check_fill1.log 2>&1; echo "check fill1 rc=$?"; tail -1 gpurun_out/s7/check_fill1.log
LLMT_WPP_FILL=1 LLMT_WPP_SLOTS=2 timeout -k 10 120 python -u bench/wgrad_pp.py check > gpurun_out/s7/check_fill1_s2.log 2>&1; echo "check fill1 slots2 rc=$?"; tail -1 gpurun_out/s7/check_fill1_s2.log
grep -c '"ok": false' gpurun_out/s7/check_fill1.log gpurun_out/s7/check_fill1_s2.log
for rnd in 1 2; do
for v in "LLMT_WPP_FILL=0" "LLMT_WPP_FILL=1" "LLMT_WPP_FILL=1 LLMT_WPP_SLOTS=2"; do
  tag=$(echo "$v" | tr -dc 'A-Z0-9=_' | tr '=' '-')
  env $v timeout -k 10 120 python -u bench/wgrad_pp.py time --tokens 131072 --only pp_slab,pp_slab_bias > gpurun_out/s7/${tag}_r$rnd.log 2>&1 || exit 1
done
done
for f in gpurun_out/s7/LLMT*.log; do echo "$f"; grep -v amdgpu "$f" | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('  ', d['gemm'], d['variant'], d['ms'], d['TFLOPs'])"; done
