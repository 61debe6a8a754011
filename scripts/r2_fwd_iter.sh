#!/usr/bin/env bash
# attention iteration: stand-alone timers (+ forward probe summary), the GPU attention tests, PMC
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/fwditer
mkdir -p $OUT
BIN=bench/native/bin
for v in ${VARIANTS:-fwd_new bwd_new}; do
  for b in 32 128; do timeout -k 10 60 $BIN/$v $b $v | tee -a $OUT/ab.log; done
done
timeout -k 10 60 $BIN/fwd_new_probe 32 probe > $OUT/probe_b32.log 2>&1
grep -E "grid|mean|qb=(0|3|7) w=(0|3)" $OUT/probe_b32.log | cut -c1-220
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_kernels_gpu.py tests/test_deterministic_gpu.py -k "attention or attn or column_sums" -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
if [ "${PMC:-0}" = 1 ]; then OUT=$OUT/pmc bash scripts/attn_pmc.sh | tee $OUT/pmc.txt; fi
