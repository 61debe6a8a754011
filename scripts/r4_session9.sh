# weight-gradient fills: DMA (0) vs register-staged 2 sets (1, 2 slots) vs 3 sets (2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/s9
LLMT_WPP_FILL=2 timeout -k 10 120 python -u bench/wgrad_pp.py check > gpurun_out/s9/check_fill2.log 2>&1; echo "check fill2 rc=$?"; grep -c '"ok": false' gpurun_out/s9/check_fill2.log
for rnd in 1 2; do
for v in "LLMT_WPP_FILL=0" "LLMT_WPP_FILL=1 LLMT_WPP_SLOTS=2" "LLMT_WPP_FILL=2"; do
  tag=$(echo "$v" | tr -dc 'A-Z0-9=_' | tr '=' '-')
  for m in 131072 32768; do
    env $v timeout -k 10 120 python -u bench/wgrad_pp.py time --tokens $m --only pp_slab,pp_slab_bias > gpurun_out/s9/${tag}_m${m}_r$rnd.log 2>&1 || exit 1
  done
done
done
for v in "LLMT_WPP_FILL=0" "LLMT_WPP_FILL=1 LLMT_WPP_SLOTS=2" "LLMT_WPP_FILL=2"; do
  tag=$(echo "$v" | tr -dc 'A-Z0-9=_' | tr '=' '-')
  env $v timeout -k 10 120 python -u bench/wgrad_pp.py time --model head --only pp_auto > gpurun_out/s9/${tag}_head.log 2>&1 || exit 1
done
for f in gpurun_out/s9/LLMT*.log; do echo "$f"; grep -v amdgpu "$f" | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('  ', d['gemm'], d['variant'], d['ms'], d['TFLOPs'])"; done
