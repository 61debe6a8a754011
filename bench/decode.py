#!/usr/bin/env python3
"""Decode latency: GPT-2 124M (bf16, random init) KV-cached greedy generation on one MI355X,
eager PyTorch ops vs the hipGraph-captured step (llmtrain.inference.graph_decode).

    python bench/decode.py [--batch 1 8] [--new-tokens 256] [--prompt 16]

Prints one JSON line per (batch, path) with ms/token and generated tokens/s.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from llmtrain.inference import generate  # noqa: E402
from llmtrain.models.gpt import GPT  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--new-tokens", type=int, default=256)
    ap.add_argument("--prompt", type=int, default=16)
    args = ap.parse_args()
    torch.manual_seed(0)
    model = GPT(vocab_size=50257, block_size=1024, d_model=768, n_layers=12, n_heads=12, d_ff=3072, dropout=0.0)
    model = model.to("cuda", torch.bfloat16).eval()
    for bsz in args.batch:
        prompt = torch.randint(0, 50257, (bsz, args.prompt), device="cuda")
        for path in ("eager", "hipgraph"):
            graph = path == "hipgraph"
            generate(model, prompt, 8, temperature=0.0, top_k=None, use_graph=graph)  # warm-up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = generate(model, prompt, args.new_tokens, temperature=0.0, top_k=None, use_graph=graph)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            n = out.shape[1] - args.prompt
            print(json.dumps({
                "bench": "decode", "model": "GPT-2 124M", "dtype": "bf16", "path": path, "batch": bsz,
                "prompt": args.prompt, "new_tokens": n, "ms_per_token": round(1e3 * dt / n, 3),
                "tokens_per_s": round(bsz * n / dt, 1),
            }), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
