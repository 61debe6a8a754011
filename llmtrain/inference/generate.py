"""Autoregressive generation for the ``gpt`` model with a KV cache.

The reference ships generation only as notebook code (notebooks/trained_vs_random_completion.ipynb,
cells ``generate_text`` and ``top_next_tokens``): each new token re-runs the WHOLE cropped context
through the model.  Here the same sampling semantics run incrementally:

* prefill once, then one token per step against per-layer K/V caches preallocated at
  ``[B, H, block_size, head_dim]`` (one allocation, no per-step concatenation);
* sampling is token-for-token the notebook's: ``temperature <= 0`` -> argmax, otherwise
  ``logits / temperature``, optional top-k cutoff (values below the k-th -> -inf), softmax,
  ``torch.multinomial``; with the same seed the cached path draws the same tokens;
* past ``block_size`` tokens the reference crops the context to the last ``block_size`` tokens,
  which RE-POSITIONS them (learned absolute positions), so a cache cannot be reused; this module
  then falls back to exactly that cropped full recompute per step.

Decode is memory-bound (the weights are streamed once per token), so it runs on PyTorch ops —
hipBLASLt GEMVs and SDPA on MI355X — in the weights' dtype, or under bf16 autocast when asked.
"""

from __future__ import annotations

import contextlib
from dataclasses import dataclass
from typing import Any

import torch
import torch.nn.functional as F

from llmtrain.models.gpt import GPT

__all__ = ["KVCache", "forward_cached", "generate", "generate_text", "sample_next_token", "top_next_tokens"]


@dataclass
class KVCache:
    """Per-layer key/value buffers ``[B, H, capacity, head_dim]`` and the filled length."""

    keys: list[torch.Tensor]
    values: list[torch.Tensor]
    length: int = 0

    @classmethod
    def allocate(cls, model: GPT, batch: int, *, dtype: torch.dtype, device: torch.device) -> KVCache:
        hd = model.d_model // model.n_heads
        shape = (batch, model.n_heads, model.block_size, hd)
        ks = [torch.empty(shape, dtype=dtype, device=device) for _ in range(model.n_layers)]
        vs = [torch.empty(shape, dtype=dtype, device=device) for _ in range(model.n_layers)]
        return cls(ks, vs, 0)

    @property
    def capacity(self) -> int:
        return self.keys[0].shape[2]


def _attend(attn: Any, x: torch.Tensor, cache: KVCache, layer: int) -> torch.Tensor:
    """Causal attention of the new positions ``x`` [B, n, d] over cache[:length] + themselves."""
    bsz, n, _ = x.shape
    heads = attn.qkv_proj(x).view(bsz, n, 3, attn.n_heads, attn.head_dim)
    q, k, v = (t.transpose(1, 2) for t in heads.unbind(dim=2))
    start = cache.length
    kc, vc = cache.keys[layer], cache.values[layer]
    kc[:, :, start : start + n] = k.to(kc.dtype)
    vc[:, :, start : start + n] = v.to(vc.dtype)
    keys, values = kc[:, :, : start + n], vc[:, :, : start + n]
    if n == 1:
        out = F.scaled_dot_product_attention(q, keys.to(q.dtype), values.to(q.dtype))
    else:
        # new query i (absolute start+i) sees keys 0..start+i
        qpos = torch.arange(start, start + n, device=x.device)[:, None]
        kpos = torch.arange(start + n, device=x.device)[None, :]
        out = F.scaled_dot_product_attention(q, keys.to(q.dtype), values.to(q.dtype), attn_mask=kpos <= qpos)
    return attn.out_proj(out.transpose(1, 2).reshape(bsz, n, attn.d_model))


@torch.no_grad()
def forward_cached(model: GPT, ids: torch.Tensor, cache: KVCache) -> torch.Tensor:
    """Logits of the last new position; appends the new tokens' K/V to ``cache``."""
    bsz, n = ids.shape
    if cache.length + n > cache.capacity:
        raise ValueError("KV cache overflow: context exceeds block_size")
    pos = torch.arange(cache.length, cache.length + n, device=ids.device)
    x = model.drop(model.token_embedding(ids) + model.position_embedding(pos)[None])
    for i, blk in enumerate(model.blocks):
        x = x + _attend(blk.attn, blk.ln_1(x), cache, i)
        x = x + blk.mlp_dropout(blk.mlp_proj(blk.mlp_act(blk.mlp_fc(blk.ln_2(x)))))
    cache.length += n
    return model.lm_head(model.ln_f(x[:, -1:]))[:, -1]


def sample_next_token(
    logits: torch.Tensor, *, temperature: float, top_k: int | None, generator: torch.Generator | None = None
) -> torch.Tensor:
    """The notebook's sampling rule on ``logits`` [B, V] -> token ids [B, 1]."""
    if temperature <= 0:
        return torch.argmax(logits, dim=-1, keepdim=True)
    logits = logits / temperature
    if top_k is not None and top_k > 0:
        k = min(top_k, logits.size(-1))
        cutoff = torch.topk(logits, k=k).values[:, -1].unsqueeze(-1)
        logits = torch.where(logits < cutoff, torch.full_like(logits, float("-inf")), logits)
    probs = torch.softmax(logits.float(), dim=-1)
    return torch.multinomial(probs, num_samples=1, generator=generator)


@torch.no_grad()
def generate(
    model: GPT,
    ids: torch.Tensor,
    max_new_tokens: int,
    *,
    temperature: float = 0.8,
    top_k: int | None = 40,
    eos_token_id: int | None = None,
    generator: torch.Generator | None = None,
    use_cache: bool = True,
    autocast_dtype: torch.dtype | None = None,
    use_graph: bool = False,
) -> torch.Tensor:
    """Extend ``ids`` [B, T0] by up to ``max_new_tokens`` sampled tokens (stops early once every
    row has produced ``eos_token_id``).  ``use_graph`` decodes through a captured hipGraph
    (:class:`llmtrain.inference.graph_decode.GraphDecoder`; GPU, weights already in the compute
    dtype, no autocast); the sampled tokens follow the same RNG stream as the eager path."""
    was_training = model.training
    model.eval()
    device = ids.device
    ctx = (
        torch.autocast(device_type=device.type, dtype=autocast_dtype)
        if autocast_dtype is not None and device.type == "cuda"
        else contextlib.nullcontext()
    )
    block = model.block_size
    out = ids
    done = torch.zeros(ids.shape[0], dtype=torch.bool, device=device)
    cache: KVCache | None = None
    decoder = None
    if use_graph and use_cache and autocast_dtype is None:
        from llmtrain.inference.graph_decode import GraphDecoder

        decoder = GraphDecoder.for_model(model, ids.shape[0])  # captured once on GPU; eager static step on CPU
        decoder.cache.length = 0
    try:
        with ctx:
            for _ in range(max_new_tokens):
                if decoder is not None and out.shape[1] <= block:
                    if decoder.length == 0:
                        logits = decoder.prefill(out).clone()
                    else:
                        logits = decoder.decode(out[:, -1:]).clone()
                elif decoder is None and use_cache and out.shape[1] <= block:
                    if cache is None:
                        dtype = model.token_embedding.weight.dtype if autocast_dtype is None else autocast_dtype
                        cache = KVCache.allocate(model, out.shape[0], dtype=dtype, device=device)
                        logits = forward_cached(model, out, cache)
                    else:
                        logits = forward_cached(model, out[:, -1:], cache)
                else:  # reference semantics past block_size: cropped, re-positioned recompute
                    logits = model(out[:, -block:])[:, -1, :]
                nxt = sample_next_token(logits.float(), temperature=temperature, top_k=top_k, generator=generator)
                if eos_token_id is not None:
                    nxt = torch.where(done[:, None], torch.full_like(nxt, eos_token_id), nxt)
                    done |= nxt[:, 0] == eos_token_id
                out = torch.cat((out, nxt), dim=1)
                if use_cache and cache is not None and out.shape[1] > block:
                    cache = None  # the next step crops and re-positions: no reusable cache
                if eos_token_id is not None and bool(done.all()):
                    break
    finally:
        model.train(was_training)
    return out


def generate_text(
    model: GPT,
    tokenizer: Any,
    prompt: str,
    max_new_tokens: int = 48,
    temperature: float = 0.8,
    top_k: int | None = 40,
    seed: int = 1234,
    *,
    use_cache: bool = True,
    use_graph: bool = False,
) -> str:
    """Notebook-compatible helper: seed, encode, generate, decode."""
    torch.manual_seed(seed)
    device = next(model.parameters()).device
    x = torch.tensor([tokenizer.encode(prompt)], dtype=torch.long, device=device)
    y = generate(
        model, x, max_new_tokens, temperature=temperature, top_k=top_k, use_cache=use_cache, use_graph=use_graph
    )
    return tokenizer.decode(y[0].tolist())


@torch.no_grad()
def top_next_tokens(model: GPT, tokenizer: Any, text: str, k: int = 10) -> list[tuple[str, float]]:
    """The ``k`` most likely next tokens after ``text`` with their probabilities."""
    was_training = model.training
    model.eval()
    device = next(model.parameters()).device
    ids = tokenizer.encode(text)[-model.block_size :]
    logits = model(torch.tensor([ids], dtype=torch.long, device=device))[:, -1, :]
    model.train(was_training)
    probs = torch.softmax(logits.float(), dim=-1)
    top_p, top_i = torch.topk(probs, k=min(k, probs.size(-1)), dim=-1)
    return [
        (tokenizer.decode([t]).replace("\n", "\\n"), float(p)) for t, p in zip(top_i[0].tolist(), top_p[0].tolist())
    ]
