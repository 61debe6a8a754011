"""Fused cross-entropy kernel alone at the LM-head shape (M rows x 50304 padded vocab, bf16).

    python bench/ce_one.py [M]
"""

from __future__ import annotations

import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from micro import timeit  # noqa: E402


def main() -> None:
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    from llmtrain.ops import _ext

    _ext.require()
    ops = torch.ops.llmtrain_hip
    V, Vp = 50257, 50304
    logits = torch.randn(M, Vp, device="cuda", dtype=torch.bfloat16)
    labels = torch.randint(0, V, (M,), device="cuda")
    roww = torch.full((M,), 1.0 / M, device="cuda")
    ms = timeit(lambda: ops.cross_entropy_fwd_bwd(logits, labels, V, roww), iters=10, warmup=3)
    gb = 2.0 * M * Vp * 2 / 1e9
    print(json.dumps({"op": "ce_fwd_bwd", "M": M, "ms": round(ms, 3), "TB/s": round(gb / ms, 2)}), flush=True)


if __name__ == "__main__":
    main()
