"""Training FLOP accounting and MFU against the MI355X dense bf16 peak.

``6·N`` (forward + backward GEMMs over all non-embedding-lookup parameters, the tied LM head
counted once as a GEMM) plus ``12·L·T·d`` for attention scores and values (full, not causal-
halved — the usual convention, SURVEY §6.4: GPT-2 124M ≈ 0.86 GFLOP/token at T=1024).
"""

from __future__ import annotations

from torch import nn

__all__ = ["MI355X_BF16_DENSE_PEAK", "mfu", "training_flops_per_token"]

MI355X_BF16_DENSE_PEAK = 2.5e15  # FLOP/s, dense (AMD's 5 PF figure includes 2:1 sparsity)


def training_flops_per_token(model: nn.Module, seq_len: int) -> float:
    n_params = sum(p.numel() for p in model.parameters())
    pos = getattr(model, "position_embedding", None)
    if pos is not None:
        n_params -= pos.weight.numel()  # a lookup, not a GEMM
    n_layers = getattr(model, "n_layers", 0)
    d_model = getattr(model, "d_model", 0)
    return 6.0 * n_params + 12.0 * n_layers * seq_len * d_model


def mfu(tokens_per_sec_per_gpu: float, flops_per_token: float, peak: float = MI355X_BF16_DENSE_PEAK) -> float:
    return tokens_per_sec_per_gpu * flops_per_token / peak
