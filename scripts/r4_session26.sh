#!/bin/bash
# weight gradients on the library (heuristics, then TunableOp-tuned) vs the ping-pong kernel
set -eo pipefail
O=gpurun_out/s26
mkdir -p $O
timeout -k 10 300 python -u bench/wgrad_library.py > $O/heuristics.txt 2>&1
( while sleep 45; do echo "tuning..."; done ) &
HB=$!
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=20 \
PYTORCH_TUNABLEOP_FILENAME=$O/wgrad_tuned%d.csv timeout -k 10 900 python -u bench/wgrad_library.py > $O/tuned.txt 2>&1 || true
kill $HB
