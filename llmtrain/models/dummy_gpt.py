"""``dummy_gpt``: tiny smoke-test model (reference ``models/dummy_gpt.py:13-90``).

Deliberately keeps the reference quirks: one bidirectional
``nn.TransformerEncoderLayer`` (no causal mask, torch defaults d_ff=2048 / dropout 0.1 / ReLU),
``d_model`` clamped to ≤ 64 and plain (unmasked) cross-entropy.
"""

from __future__ import annotations

from typing import Any

import torch
import torch.nn.functional as F
from torch import nn

from llmtrain.config.schemas import RunConfig
from llmtrain.models.base import LazyFloat, ModelAdapter, validate_lm_batch
from llmtrain.registry.models import register_model

__all__ = ["DummyGPTAdapter"]


class _TinyGPT(nn.Module):
    def __init__(self, vocab_size: int, d_model: int, n_heads: int) -> None:
        super().__init__()
        self.embed = nn.Embedding(vocab_size, d_model)
        layer = nn.TransformerEncoderLayer(d_model=d_model, nhead=n_heads, batch_first=True)
        self.encoder = nn.TransformerEncoder(layer, num_layers=1, enable_nested_tensor=False)
        self.lm_head = nn.Linear(d_model, vocab_size, bias=False)

    def forward(self, input_ids: torch.Tensor, attention_mask: torch.Tensor | None = None) -> torch.Tensor:
        pad = None if attention_mask is None else attention_mask == 0
        return self.lm_head(self.encoder(self.embed(input_ids), src_key_padding_mask=pad))


def _pick_heads(d_model: int, requested: int) -> int:
    heads = max(1, min(requested, d_model))
    if d_model % heads:
        heads = 2 if d_model % 2 == 0 else 1
    return heads


@register_model("dummy_gpt")
class DummyGPTAdapter(ModelAdapter):
    def build_model(self, cfg: RunConfig) -> nn.Module:
        d_model = min(cfg.model.d_model or 128, 64)
        return _TinyGPT(cfg.model.vocab_size or 128, d_model, _pick_heads(d_model, cfg.model.n_heads))

    def build_tokenizer(self, cfg: RunConfig) -> Any | None:
        return None

    def compute_loss(
        self, model: nn.Module, batch: dict[str, torch.Tensor]
    ) -> tuple[torch.Tensor, dict[str, float]]:
        validate_lm_batch(batch)
        logits = model(batch["input_ids"], attention_mask=batch.get("attention_mask"))
        loss = F.cross_entropy(logits.reshape(-1, logits.size(-1)).float(), batch["labels"].reshape(-1))
        return loss, {"loss": LazyFloat(loss)}
