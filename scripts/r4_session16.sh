#!/bin/bash
# wgrad ping-pong kernel: per-phase cycle split (s_memtime probe, LLMT_WPP_SKEL=9)
set -eo pipefail
mkdir -p gpurun_out/s16
export LLMT_WPP_SKEL=9
for g in qkv fc proj out head; do
  timeout -k 10 120 python -u bench/wgrad_pp.py probe --gemm $g >> gpurun_out/s16/probe.txt 2>&1
done
unset LLMT_WPP_SKEL
timeout -k 10 120 python -u bench/wgrad_pp.py time --only pp_slab >> gpurun_out/s16/time.txt 2>&1
