"""One weight-gradient GEMM shape, repeated (for rocprofv3 counter passes).

    python bench/wgrad_one.py N K M [reps] [tile] [split]
"""

from __future__ import annotations

import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main() -> None:
    a = [int(v) for v in sys.argv[1:]]
    N, K, M = a[0], a[1], a[2]
    reps = a[3] if len(a) > 3 else 5
    tile = a[4] if len(a) > 4 else 0
    split = a[5] if len(a) > 5 else 0
    from llmtrain.ops import _ext

    _ext.require()
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    acc = torch.zeros(N, K, device="cuda")
    for _ in range(reps):
        torch.ops.llmtrain_hip.wgrad_gemm(dy, x, acc, split, tile)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        torch.ops.llmtrain_hip.wgrad_gemm(dy, x, acc, split, tile)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    print(f"wgrad N={N} K={K} M={M} tile={tile} split={split}: {ms:.4f} ms {2.0 * M * N * K / ms / 1e9:.1f} TF")


if __name__ == "__main__":
    main()
