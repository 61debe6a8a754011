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
# attention backward: static priority for waves 4-7 (LLMT_ATTN_BWD_PRIO)
for r in 1 2; do
  for pr in 0 1; do
    LLMT_ATTN_BWD_PRIO=$pr timeout -k 10 120 python -u bench/micro.py attn 128 2>&1 | grep "llmtrain" | sed "s/^/prio$pr /" >> $O/attn_prio.txt
  done
done
# forward GEMM ping-pong kernel: numerics, then timing vs hipBLASLt / gemm_fused, both fill schedules
timeout -k 10 180 python -u bench/gemm_pp.py check > $O/gpp_check.txt 2>&1
LLMT_GPP_FILL=1 timeout -k 10 180 python -u bench/gemm_pp.py check > $O/gpp_check_fill1.txt 2>&1
for r in 1 2; do
  timeout -k 10 180 python -u bench/gemm_pp.py time 2>&1 | grep TFLOPs | sed "s/^/fill3 /" >> $O/gpp_time.txt
  LLMT_GPP_FILL=1 timeout -k 10 180 python -u bench/gemm_pp.py time --only pp,pp_gelu 2>&1 | grep TFLOPs | sed "s/^/fill1 /" >> $O/gpp_time.txt
done
# step A/B: forward GEMMs on the ping-pong kernel (only if its numerics passed)
if ! grep -q '"ok": false' $O/gpp_check.txt && grep -q '"ok": true' $O/gpp_check.txt; then
  bash scripts/abn.sh "LLMTRAIN_GEMM_PP=none" "LLMTRAIN_GEMM_PP=fwd,fwd_gelu" "LLMTRAIN_GEMM_PP=dx_gelu,dx_attn" "LLMTRAIN_GEMM_PP=all" -- --steps 10 --warmup 3 > $O/ab_gemm_pp_mb128.txt 2>&1
fi
