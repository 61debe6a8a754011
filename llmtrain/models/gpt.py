"""Decoder-only pre-LN GPT (the ``"gpt"`` adapter) — MI355X build.

Module tree, parameter names/shapes, initialisation and the persistent ``causal_mask`` buffer
match the reference (``models/gpt.py:15-184``), so ``state_dict`` checkpoints are interchangeable:

    token_embedding, position_embedding, drop, blocks[i].{ln_1, attn.{qkv_proj, out_proj,
    causal_mask}, ln_2, mlp_fc, mlp_proj}, ln_f, lm_head (weight tied to token_embedding)

Two execution paths share these parameters:

* **module path** (``GPT.forward``) — ordinary autograd over PyTorch ops; used on CPU, for fp32
  runs and as the parity oracle in tests;
* **fused path** (``GPT.fused_loss``) — the hand-scheduled MI355X engine in
  :mod:`llmtrain.models.gpt_engine`: bf16 GEMMs on flat shadow weights, gfx950 HIP kernels for
  embedding / add+LayerNorm / flash attention / GELU / fused cross-entropy, a hand-written
  backward that accumulates fp32 gradients in place and releases data-parallel gradient buckets
  as soon as each layer's gradients are final.
"""

from __future__ import annotations

import math
from typing import Any

import torch
import torch.nn.functional as F
from torch import nn

from llmtrain.config.schemas import RunConfig
from llmtrain.models.base import LazyFloat, ModelAdapter, validate_lm_batch
from llmtrain.registry.models import register_model

__all__ = ["GPT", "CausalSelfAttention", "GPTAdapter", "TransformerBlock"]


class CausalSelfAttention(nn.Module):
    """Multi-head causal self-attention with a packed QKV projection."""

    def __init__(self, d_model: int, n_heads: int, block_size: int, dropout: float) -> None:
        super().__init__()
        if d_model % n_heads:
            raise ValueError("d_model must be divisible by n_heads")
        self.d_model = d_model
        self.n_heads = n_heads
        self.head_dim = d_model // n_heads
        self.dropout_p = dropout
        self.qkv_proj = nn.Linear(d_model, 3 * d_model)
        self.attn_dropout = nn.Dropout(dropout)
        self.out_proj = nn.Linear(d_model, d_model)
        self.resid_dropout = nn.Dropout(dropout)
        upper = torch.ones(block_size, block_size, dtype=torch.bool).triu(diagonal=1)
        # Persistent so checkpoints carry ``blocks.{i}.attn.causal_mask`` like the reference.
        self.register_buffer("causal_mask", upper[None, None])

    def forward(self, x: torch.Tensor, attention_mask: torch.Tensor | None = None) -> torch.Tensor:
        bsz, seqlen, _ = x.shape
        block = self.causal_mask.shape[-1]
        if seqlen > block:
            raise ValueError(f"Input sequence length {seqlen} exceeds block size {block}.")
        if attention_mask is not None and attention_mask.shape != (bsz, seqlen):
            raise ValueError(
                "Expected attention_mask to have shape (B, T); "
                f"got {tuple(attention_mask.shape)} for {(bsz, seqlen)}."
            )
        heads = self.qkv_proj(x).view(bsz, seqlen, 3, self.n_heads, self.head_dim)
        q, k, v = (t.transpose(1, 2) for t in heads.unbind(dim=2))

        keep = None if attention_mask is None else attention_mask.bool()
        if keep is None and x.device.type == "cuda":
            out = F.scaled_dot_product_attention(
                q, k, v, is_causal=True, dropout_p=self.dropout_p if self.training else 0.0
            )
        else:
            scores = (q @ k.transpose(-2, -1)) / math.sqrt(self.head_dim)
            floor = torch.finfo(scores.dtype).min
            scores = scores.masked_fill(self.causal_mask[:, :, :seqlen, :seqlen], floor)
            if keep is not None:
                scores = scores.masked_fill(~keep[:, None, None, :], floor)
            out = self.attn_dropout(torch.softmax(scores, dim=-1)) @ v
        out = self.resid_dropout(self.out_proj(out.transpose(1, 2).reshape(bsz, seqlen, self.d_model)))
        if keep is not None:
            out = out * keep[:, :, None].to(out.dtype)
        return out


class TransformerBlock(nn.Module):
    """Pre-norm block: ``x + attn(ln_1(x))`` then ``x + mlp(ln_2(x))``."""

    def __init__(self, d_model: int, n_heads: int, d_ff: int, block_size: int, dropout: float) -> None:
        super().__init__()
        self.ln_1 = nn.LayerNorm(d_model)
        self.attn = CausalSelfAttention(d_model, n_heads, block_size, dropout)
        self.ln_2 = nn.LayerNorm(d_model)
        self.mlp_fc = nn.Linear(d_model, d_ff)
        self.mlp_act = nn.GELU()
        self.mlp_proj = nn.Linear(d_ff, d_model)
        self.mlp_dropout = nn.Dropout(dropout)

    def forward(self, x: torch.Tensor, attention_mask: torch.Tensor | None = None) -> torch.Tensor:
        x = x + self.attn(self.ln_1(x), attention_mask=attention_mask)
        return x + self.mlp_dropout(self.mlp_proj(self.mlp_act(self.mlp_fc(self.ln_2(x)))))


class GPT(nn.Module):
    """GPT-2 style language model; see the module docstring for the two execution paths."""

    def __init__(
        self,
        vocab_size: int,
        block_size: int,
        d_model: int,
        n_layers: int,
        n_heads: int,
        d_ff: int,
        dropout: float,
        tie_embeddings: bool = True,
    ) -> None:
        super().__init__()
        self.vocab_size = vocab_size
        self.block_size = block_size
        self.d_model = d_model
        self.n_layers = n_layers
        self.n_heads = n_heads
        self.d_ff = d_ff
        self.dropout = dropout
        self.tie_embeddings = tie_embeddings

        self.token_embedding = nn.Embedding(vocab_size, d_model)
        self.position_embedding = nn.Embedding(block_size, d_model)
        self.drop = nn.Dropout(dropout)
        self.blocks = nn.ModuleList(
            TransformerBlock(d_model, n_heads, d_ff, block_size, dropout) for _ in range(n_layers)
        )
        self.ln_f = nn.LayerNorm(d_model)
        self.lm_head = nn.Linear(d_model, vocab_size, bias=False)
        if tie_embeddings:
            self.lm_head.weight = self.token_embedding.weight
        self._reset_parameters()
        self._engine: Any = None  # llmtrain.models.gpt_engine.FusedGPTEngine once prepared

    # -- initialisation (reference gpt.py:148-165) ----------------------------------------

    def _reset_parameters(self) -> None:
        for module in self.modules():
            if isinstance(module, (nn.Linear, nn.Embedding)):
                nn.init.normal_(module.weight, mean=0.0, std=0.02)
                if isinstance(module, nn.Linear) and module.bias is not None:
                    nn.init.zeros_(module.bias)
        resid_std = 0.02 / math.sqrt(2 * self.n_layers)
        for block in self.blocks:
            nn.init.normal_(block.attn.out_proj.weight, mean=0.0, std=resid_std)
            nn.init.normal_(block.mlp_proj.weight, mean=0.0, std=resid_std)

    # -- module path -----------------------------------------------------------------------

    def forward(self, input_ids: torch.Tensor, attention_mask: torch.Tensor | None = None) -> torch.Tensor:
        _, seqlen = input_ids.shape
        if seqlen > self.block_size:
            raise ValueError(f"Input sequence length {seqlen} exceeds block size {self.block_size}.")
        pos = torch.arange(seqlen, device=input_ids.device)
        x = self.drop(self.token_embedding(input_ids) + self.position_embedding(pos)[None])
        for block in self.blocks:
            x = block(x, attention_mask=attention_mask)
        return self.lm_head(self.ln_f(x))

    # -- fused path ------------------------------------------------------------------------

    def fused_supported(self, device_type: str = "cuda") -> bool:
        """Whether the fused engine covers this shape on ``device_type``.  On the GPU the
        flash-attention kernels take head dims that are multiples of 8 up to 64 (64 is the fast
        specialisation — GPT-2 124M and XL; the reference presets' 32 and 48 run zero-filled in
        the same tiles) or exactly 128 (two 64-wide halves; a 4-wave one-wave-per-
        SIMD backward) and key-padding masks; LayerNorm widths need d % 4 == 0,
        d <= 2048.  Other shapes train on the module path.  On CPU the engine runs the reference
        ops, which take any shape.  Dropout is supported everywhere (counter-based masks fused into
        the embedding, add+LayerNorm and flash-attention kernels)."""
        if device_type != "cuda":
            return True
        if self.d_model % self.n_heads != 0:
            return False
        hd = self.d_model // self.n_heads
        return (
            ((hd % 8 == 0 and 8 <= hd <= 64) or hd == 128)
            and self.d_model % 4 == 0
            and self.d_model <= 2048
            and self.d_ff % 8 == 0
        )

    def prepare_runtime(
        self, *, compute_dtype: torch.dtype = torch.bfloat16, residual: str | None = None, mlp_store: str | None = None
    ) -> Any:
        """Move parameters into flat buffers and build the fused engine (idempotent).

        Call after ``model.to(device)`` and before building the optimizer.  ``residual``: storage
        of the residual stream and its gradient (``model.extra.residual_dtype``; None = bf16 with
        the bf16 compute dtype, fp32 otherwise — see :class:`~llmtrain.models.gpt_engine.FusedGPTEngine`).
        """
        if self._engine is None:
            from llmtrain.models.gpt_engine import FusedGPTEngine

            self._engine = FusedGPTEngine(self, compute_dtype=compute_dtype, residual=residual, mlp_store=mlp_store)
        return self._engine

    @property
    def engine(self) -> Any:
        return self._engine

    @property
    def flat_store(self) -> Any:
        return None if self._engine is None else self._engine.store

    def fused_loss(
        self,
        input_ids: torch.Tensor,
        labels: torch.Tensor,
        attention_mask: torch.Tensor | None = None,
    ) -> torch.Tensor:
        """Mean (masked) next-token loss computed by the fused engine; ``.backward()`` on the
        result runs the hand-written backward."""
        if self._engine is None:
            raise RuntimeError("call prepare_runtime() before fused_loss()")
        if input_ids.shape[1] > self.block_size:
            raise ValueError(
                f"Input sequence length {input_ids.shape[1]} exceeds block size {self.block_size}."
            )
        return self._engine.loss(input_ids, labels, attention_mask)


def _resolve_vocab(cfg: RunConfig, adapter: GPTAdapter) -> int:
    if cfg.model.vocab_size is not None:
        return cfg.model.vocab_size
    tokenizer = adapter.build_tokenizer(cfg)
    n_vocab = getattr(tokenizer, "n_vocab", None)
    if not isinstance(n_vocab, int) or n_vocab <= 0:
        raise ValueError("GPT tokenizer must expose a positive integer n_vocab.")
    return n_vocab


@register_model("gpt")
class GPTAdapter(ModelAdapter):
    """Adapter for :class:`GPT`. Chooses the fused engine when the model was prepared for it."""

    def build_model(self, cfg: RunConfig) -> nn.Module:
        m = cfg.model
        return GPT(
            vocab_size=_resolve_vocab(cfg, self),
            block_size=m.block_size,
            d_model=m.d_model,
            n_layers=m.n_layers,
            n_heads=m.n_heads,
            d_ff=m.d_ff,
            dropout=m.dropout,
            tie_embeddings=m.tie_embeddings,
        )

    def build_tokenizer(self, cfg: RunConfig) -> Any | None:
        from llmtrain.data.tokenizer import get_gpt2_tokenizer

        return get_gpt2_tokenizer()

    def compute_loss(
        self, model: nn.Module, batch: dict[str, torch.Tensor]
    ) -> tuple[torch.Tensor, dict[str, float]]:
        validate_lm_batch(batch, min_len=2)
        input_ids, labels = batch["input_ids"], batch["labels"]
        mask = batch.get("attention_mask")
        core = getattr(model, "module", model)
        if isinstance(core, GPT) and core.engine is not None:
            # ``model`` may be a data-parallel wrapper whose fused_loss arms the grad reducer.
            loss = model.fused_loss(input_ids, labels, mask)
            return loss, {"loss": LazyFloat(loss)}

        logits = model(input_ids, attention_mask=mask)
        per_token = F.cross_entropy(
            logits.reshape(-1, logits.size(-1)).float(), labels.reshape(-1), reduction="none"
        )
        if mask is None:
            loss = per_token.mean()
        else:
            keep = mask.reshape(-1).bool()
            if not bool(keep.any()):
                raise ValueError("attention_mask has no valid target tokens.")
            loss = per_token[keep].mean()
        return loss, {"loss": LazyFloat(loss)}
