#!/bin/bash
# wgrad ping-pong: fills inside the MFMA segment (LLMT_WPP_FILL=3) vs register-staged in LOAD (1)
set -eo pipefail
mkdir -p gpurun_out/s17
O=gpurun_out/s17
LLMT_WPP_FILL=3 timeout -k 10 180 python -u bench/wgrad_pp.py check > $O/check_fill3.txt 2>&1
LLMT_WPP_FILL=3 LLMT_WPP_PLACE=1 timeout -k 10 180 python -u bench/wgrad_pp.py check > $O/check_fill3_p1.txt 2>&1
for cfg in "1 0" "3 0" "3 1"; do
  set -- $cfg
  for g in qkv fc head; do
    LLMT_WPP_SKEL=9 LLMT_WPP_FILL=$1 LLMT_WPP_PLACE=$2 timeout -k 10 120 python -u bench/wgrad_pp.py probe --gemm $g 2>&1 | grep gemm | sed "s/^/fill$1 place$2 /" >> $O/probe.txt
  done
done
for r in 1 2; do
  for cfg in "1 0" "3 0" "3 1"; do
    set -- $cfg
    LLMT_WPP_FILL=$1 LLMT_WPP_PLACE=$2 timeout -k 10 120 python -u bench/wgrad_pp.py time --only pp_slab,pp_auto 2>&1 | grep TFLOPs | sed "s/^/fill$1 place$2 /" >> $O/time.txt
    LLMT_WPP_FILL=$1 LLMT_WPP_PLACE=$2 timeout -k 10 120 python -u bench/wgrad_pp.py time --model head --only pp_auto 2>&1 | grep TFLOPs | sed "s/^/fill$1 place$2 /" >> $O/time.txt
  done
done
