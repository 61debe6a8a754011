#!/bin/bash
# weight gradients with ds_write_addtid_b32 fills (LLMT_WPP_FILL=4) vs ds_write_b128 (1)
set -eo pipefail
O=gpurun_out/s35
mkdir -p $O
LLMT_WPP_FILL=4 timeout -k 10 180 python -u bench/wgrad_pp.py check > $O/check_fill4.txt 2>&1
if grep -q '"ok": false' $O/check_fill4.txt; then echo "numerics failed"; exit 1; fi
for r in 1 2; do
  for f in 1 4; do
    LLMT_WPP_FILL=$f timeout -k 10 120 python -u bench/wgrad_pp.py time --only pp_auto 2>&1 | grep TFLOPs | sed "s/^/fill$f /" >> $O/time.txt
    LLMT_WPP_FILL=$f timeout -k 10 120 python -u bench/wgrad_pp.py time --model head --only pp_auto 2>&1 | grep TFLOPs | sed "s/^/fill$f /" >> $O/time.txt
  done
done
bash scripts/abn.sh "LLMT_WPP_FILL=1" "LLMT_WPP_FILL=4" -- --steps 10 --warmup 3 > $O/ab_mb128.txt 2>&1
bash scripts/abn.sh "LLMT_WPP_FILL=1" "LLMT_WPP_FILL=4" -- --micro-batch 32 --steps 20 --warmup 5 > $O/ab_mb32.txt 2>&1
