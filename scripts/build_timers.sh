#!/usr/bin/env bash
# Build the stand-alone attention timers (bench/native/*_timer.cpp) into bench/native/bin on the CPU
# host (hipcc cross-compiles gfx950); they travel to the GPU box with the tree.
#   fwd_new / bwd_new        : the current csrc kernels
#   fwd_new_probe / bwd_new_probe : with the per-step s_memtime probe (-DLLMT_ATTN_PROBE)
set -euo pipefail
cd "$(dirname "$0")/.."
BIN=bench/native/bin
mkdir -p "$BIN"
HIPCC="${ROCM_PATH:-/opt/rocm}/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc -x hip"
$HIPCC bench/native/attn_fwd_timer.cpp csrc/attention_fwd.hip -o $BIN/fwd_new &
$HIPCC -DLLMT_ATTN_PROBE bench/native/attn_fwd_timer.cpp csrc/attention_fwd.hip -o $BIN/fwd_new_probe &
$HIPCC bench/native/attn_bwd_timer.cpp csrc/attention_bwd.hip csrc/reduce.hip -o $BIN/bwd_new &
$HIPCC -DLLMT_ATTN_PROBE bench/native/attn_bwd_timer.cpp csrc/attention_bwd.hip csrc/reduce.hip -o $BIN/bwd_new_probe &
wait
ls -la $BIN
