"""Weight-gradient GEMMs on the library vs the ping-pong kernel, with and without TunableOp tuning.

    python bench/wgrad_library.py [M]
    PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=... python bench/wgrad_library.py

Variants per shape: addmm_fp32 (dW += dy^T x with an fp32 output matrix), mm_bf16_add (bf16 GEMM +
fp32 add), pp (csrc/gemm_wgrad_pp.hip).  One JSON line each: ms (median of 20), TFLOP/s.
"""

from __future__ import annotations

import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from micro import timeit  # noqa: E402

SHAPES = {"qkv": (2304, 768), "out": (768, 768), "fc": (3072, 768), "proj": (768, 3072), "head": (50304, 768)}


def main() -> int:
    from llmtrain.ops import _ext

    _ext.require()
    ops = torch.ops.llmtrain_hip
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    for name, (N, K) in SHAPES.items():
        dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        acc = torch.zeros(N, K, device="cuda")
        flops = 2.0 * M * N * K
        variants = {
            "addmm_fp32": lambda: torch.addmm(acc, dy.t(), x, out_dtype=torch.float32, out=acc),
            "mm_bf16_add": lambda: acc.add_(torch.mm(dy.t(), x)),
            "pp": lambda: ops.wgrad_gemm_pp(dy, x, acc, None, 0, -1),
        }
        for label, fn in variants.items():
            try:
                ms = timeit(fn)
            except RuntimeError as e:  # a variant the backend does not offer
                print(json.dumps({"gemm": name, "variant": label, "error": str(e)[:120]}), flush=True)
                continue
            print(json.dumps({"M": M, "gemm": name, "variant": label, "ms": round(ms, 4),
                              "TFLOPs": round(flops / ms / 1e9, 1)}), flush=True)
        del dy, x, acc
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
