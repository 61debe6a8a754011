#!/usr/bin/env python3
"""Build a small GPT, print parameter counts and run one forward (reference notebook
notebooks/gpt_model_smoke.ipynb; its anchor: 118,528 parameters for this config).

On a MI355X it additionally runs the fused engine (hand-written gfx950 kernels, bf16) on the same
model (head_dim 16 runs zero-filled in the 64-wide flash-attention tiles) and reports the loss gap
against the module path on the same weights.

    python examples/gpt_model_smoke.py [--device cuda]
"""

from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from llmtrain.models.gpt import GPT  # noqa: E402

CFG = {"vocab_size": 256, "block_size": 32, "d_model": 64, "n_layers": 2, "n_heads": 4, "d_ff": 256,
       "dropout": 0.1, "tie_embeddings": True}


def main(argv: list[str] | None = None) -> dict:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    args = ap.parse_args(argv)
    torch.manual_seed(7)
    model = GPT(**CFG)
    total = sum(p.numel() for p in model.parameters())
    trainable = sum(p.numel() for p in model.parameters() if p.requires_grad)
    ids = torch.randint(0, CFG["vocab_size"], (2, 16), dtype=torch.long)
    mask = torch.ones_like(ids)
    with torch.no_grad():
        logits = model(input_ids=ids, attention_mask=mask)
    info = {
        "total_parameters": total,
        "trainable_parameters": trainable,
        "logits_shape": tuple(logits.shape),
        "contains_nan": bool(torch.isnan(logits).any()),
        "token_embedding_params": model.token_embedding.weight.numel(),
        "weights_tied": model.lm_head.weight.data_ptr() == model.token_embedding.weight.data_ptr(),
        "blocks": len(model.blocks),
    }
    if args.device == "cuda":
        fused = GPT(**{**CFG, "dropout": 0.0}).cuda()
        assert fused.fused_supported("cuda")
        ref_loss = F.cross_entropy(fused(ids.cuda()).float().reshape(-1, CFG["vocab_size"]), ids.cuda().reshape(-1))
        fused.prepare_runtime(compute_dtype=torch.bfloat16)
        with torch.no_grad():
            loss = fused.fused_loss(ids.cuda(), ids.cuda())
        info["fused_minus_module_loss"] = float(loss - ref_loss)
    for k, v in info.items():
        print(f"{k}: {v:,}" if isinstance(v, int) and not isinstance(v, bool) else f"{k}: {v}")
    return info


if __name__ == "__main__":
    main()
