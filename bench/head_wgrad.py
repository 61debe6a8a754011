#!/usr/bin/env python3
"""LM-head weight gradient variants at the bench shape (GPT-2 vocab, d 768, M tokens):

    python bench/head_wgrad.py [M]

  * addmm_fp32: ``dW(fp32) += dlogits^T hf`` via ``addmm(out_dtype=fp32)`` (the engine's default)
  * mm_bf16_add: bf16-output GEMM (TunableOp-eligible) + fp32 add (torch autocast numerics)
  * wgrad_hip:   the weight-gradient kernel (csrc/gemm_wgrad_pp.hip) into dW (the engine's choice)
  * hfT_mm_fp32 / hfT_mm_bf16: dW^T = hf^T dlogits with hf^T materialised (K-contiguous A, the
    "NN" class hipBLASLt runs at ~1.7 PF for the head dX), fp32 / bf16 output, + transpose-add
Prints ms and PFLOP/s per variant, and the max error of each against an fp64-accumulated check
on a row slice.
"""

from __future__ import annotations

import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from llmtrain import ops  # noqa: E402
from llmtrain.models.gpt_engine import accumulate_wgrad  # noqa: E402
from llmtrain.runtime.tuning import enable_tuned_gemms  # noqa: E402


def timeit(fn, iters: int = 10, warmup: int = 3) -> float:
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main() -> int:
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    V, Vp, d = 50257, 50304, 768
    dev = torch.device("cuda")
    enable_tuned_gemms(dev)
    g = torch.Generator(device="cuda").manual_seed(0)
    dlogits = (torch.randn(M, Vp, device=dev, generator=g) * 1e-3).to(torch.bfloat16)
    dlogits[:, V:] = 0
    hf = torch.randn(M, d, device=dev, generator=g).to(torch.bfloat16)
    dy = dlogits[:, :V]
    flops = 2.0 * M * V * d
    ref = (dy[:, :256].double().t() @ hf.double()).float()  # first 256 vocab rows
    out = {}

    dw = torch.zeros(V, d, device=dev)
    hfT = hf.t().contiguous()
    variants = {
        "addmm_fp32": lambda: accumulate_wgrad(dw, dy, hf),
        "mm_bf16_add": lambda: dw.add_(torch.mm(dy.t(), hf)),
        "wgrad_hip": lambda: ops.wgrad_accum(dw, dy, hf),
        "hfT_mm_fp32": lambda: dw.add_(torch.mm(hf.t().contiguous(), dy, out_dtype=torch.float32).t()),
        "hfT_mm_bf16": lambda: dw.add_(torch.mm(hf.t().contiguous(), dy).t()),
        "hfT_only_mm_bf16": lambda: torch.mm(hfT, dlogits),
    }
    for name, fn in variants.items():
        dw.zero_()
        fn()
        torch.cuda.synchronize()
        err = (dw[:256] - ref).abs().max().item() / ref.abs().max().item() if name != "hfT_only_mm_bf16" else 0.0
        ms = timeit(fn, iters=10, warmup=3)
        out[name] = {"ms": round(ms, 3), "PFLOPs": round(flops / ms / 1e12, 3), "rel_err_max": err}
        print(json.dumps({"M": M, "variant": name, **out[name]}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
