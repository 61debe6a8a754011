"""Weight-gradient GEMM: llmtrain tile 128 / 256 / auto vs hipBLASLt on a model's shapes.

    python bench/wgrad_shapes.py --model gpt2-xl --tokens 16384
"""

from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from micro import timeit  # noqa: E402

SHAPES = {
    "gpt2-124m": {"qkv": (2304, 768), "out": (768, 768), "fc": (3072, 768), "proj": (768, 3072)},
    "gpt2-xl": {"qkv": (4800, 1600), "out": (1600, 1600), "fc": (6400, 1600), "proj": (1600, 6400)},
}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-xl", choices=sorted(SHAPES))
    ap.add_argument("--tokens", type=int, default=16384)
    args = ap.parse_args()
    from llmtrain.ops import _ext

    _ext.require()
    M = args.tokens
    for name, (N, K) in SHAPES[args.model].items():
        dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        acc = torch.zeros(N, K, device="cuda")
        flops = 2.0 * M * N * K
        for label, fn in {
            "auto": lambda: torch.ops.llmtrain_hip.wgrad_gemm(dy, x, acc, 0, 0),
            "tile128": lambda: torch.ops.llmtrain_hip.wgrad_gemm(dy, x, acc, 0, 128),
            "tile256": lambda: torch.ops.llmtrain_hip.wgrad_gemm(dy, x, acc, 0, 256),
            "hipblaslt": lambda: torch.addmm(acc, dy.t(), x, out_dtype=torch.float32, out=acc),
        }.items():
            ms = timeit(fn)
            print(json.dumps({"model": args.model, "M": M, "gemm": name, "variant": label, "ms": round(ms, 4),
                              "TFLOPs": round(flops / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
