"""LM head + fused cross-entropy, whole micro-batch vs row chunks small enough for the logits
chunk to stay in the 256 MiB Infinity Cache between the GEMM that writes it and the CE kernel
that overwrites it with dlogits.

    python bench/head_chunk.py --tokens 131072 --chunks 0,1024,1536,2048,4096,16384
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


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=131072)
    ap.add_argument("--chunks", default="0,1024,1536,2048,4096,16384")
    ap.add_argument("--d", type=int, default=768)
    args = ap.parse_args()
    from llmtrain.ops import _ext

    _ext.require()
    ops = torch.ops.llmtrain_hip
    M, d, V, Vp = args.tokens, args.d, 50257, 50304
    torch.manual_seed(0)
    hf = torch.randn(M, d, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(Vp, d, device="cuda") * 0.02).to(torch.bfloat16)
    labels = torch.randint(0, V, (M,), device="cuda")
    row_w = torch.full((M,), 1.0 / M, device="cuda")
    logits = torch.empty(M, Vp, device="cuda", dtype=torch.bfloat16)
    ref_rows = None
    for c in [int(x) for x in args.chunks.split(",")]:
        step = M if c <= 0 else c

        def run() -> torch.Tensor:
            outs = []
            for r0 in range(0, M, step):
                r1 = min(M, r0 + step)
                lc = logits[r0:r1]
                torch.mm(hf[r0:r1], w.t(), out=lc)
                outs.append(ops.cross_entropy_fwd_bwd(lc, labels[r0:r1], V, row_w[r0:r1]))
            return torch.cat(outs)

        rows = run()
        if ref_rows is None:
            ref_rows = rows
        err = float((rows - ref_rows).abs().max())
        ms = timeit(run, iters=10, warmup=3)
        gemm_ms = timeit(lambda: [torch.mm(hf[r0:r0 + step], w.t(), out=logits[r0:r0 + step])
                                  for r0 in range(0, M, step)], iters=10, warmup=3)
        print(json.dumps({"chunk": step, "ms_gemm_ce": round(ms, 3), "ms_gemm_only": round(gemm_ms, 3),
                          "ms_ce_est": round(ms - gemm_ms, 3), "max_abs_diff": err}), flush=True)


if __name__ == "__main__":
    main()
