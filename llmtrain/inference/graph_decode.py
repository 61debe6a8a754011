"""Single-token decode captured in a hipGraph (``torch.cuda.CUDAGraph`` is hipGraph on ROCm).

Decode of a small GPT is launch-bound, not bandwidth-bound: one GPT-2 124M token is ~150 kernel
launches (embedding, 12 x (LN, qkv GEMV, cache write, attention, out GEMV, LN, fc GEMV, GELU,
proj GEMV, adds), head GEMV) of a few microseconds each, so the host issue rate sets the
per-token latency.  :class:`GraphDecoder` records the whole step once and replays it with one
``hipGraphLaunch`` per token:

* every shape is static: the token buffer ``[B, 1]``, the position as a DEVICE scalar, the
  per-layer K/V caches ``[B, H, block_size, hd]`` (shared with the eager prefill path), and the
  logits output;
* the new K/V rows go to cache slot ``pos`` with ``index_copy_`` on the device-side index, and
  attention runs over the full cache capacity with the slots ``> pos`` masked to ``-inf``, so
  the graph is valid for every position (the masked slots contribute exact zeros);
* sampling stays outside the graph (``torch.multinomial`` draws from the caller's generator), so
  the sampled tokens follow the same RNG stream as the eager KV-cached path.

Reference behaviour this serves: notebooks/trained_vs_random_completion.ipynb ``generate_text``
(full-context recompute per token); the prefill, crop and sampling semantics are those of
:mod:`llmtrain.inference.generate`.  On CPU (no graphs) :meth:`GraphDecoder.decode` runs the same
static-shape step eagerly, which is how its numerics are tested without a GPU.
"""

from __future__ import annotations

import weakref

import torch

from llmtrain.inference.generate import KVCache, forward_cached
from llmtrain.models.gpt import GPT

__all__ = ["GraphDecoder"]

_DECODERS: weakref.WeakKeyDictionary = weakref.WeakKeyDictionary()


class GraphDecoder:
    """Prefill eagerly, then decode one token per row per call through a captured hipGraph."""

    def __init__(self, model: GPT, batch: int, *, use_graph: bool | None = None) -> None:
        self.model = model
        p = next(model.parameters())
        self.device = p.device
        self.dtype = p.dtype
        self.batch = batch
        self.cache = KVCache.allocate(model, batch, dtype=self.dtype, device=self.device)
        for buf in (*self.cache.keys, *self.cache.values):
            buf.zero_()  # masked slots are multiplied by exact zeros: they must not hold NaN/Inf
        self.tok = torch.zeros(batch, 1, dtype=torch.long, device=self.device)
        self.pos = torch.zeros(1, dtype=torch.long, device=self.device)
        self._slots = torch.arange(self.cache.capacity, device=self.device)
        self.use_graph = self.device.type == "cuda" if use_graph is None else use_graph
        if self.use_graph and self.device.type != "cuda":
            raise ValueError("hipGraph decode needs a GPU model")
        self.graph: torch.cuda.CUDAGraph | None = None
        self.logits: torch.Tensor | None = None

    @classmethod
    def for_model(cls, model: GPT, batch: int) -> GraphDecoder:
        """A decoder cached per (model, batch): the graph is captured once and replayed by every
        later ``generate`` call.  The graph reads the parameters in place, so in-place weight
        updates are seen; a model moved to another device/dtype gets a fresh decoder."""
        p = next(model.parameters())
        key = (batch, p.device, p.dtype, p.data_ptr())
        per_model = _DECODERS.setdefault(model, {})
        dec = per_model.get(key)
        if dec is None:
            per_model.clear()  # stale keys hold caches of a previous placement
            dec = per_model[key] = cls(model, batch)
        return dec

    @property
    def length(self) -> int:
        return self.cache.length

    # -- eager pieces ----------------------------------------------------------------------

    @torch.no_grad()
    def prefill(self, ids: torch.Tensor) -> torch.Tensor:
        """Run the prompt ``[B, T0]`` through the model, filling the cache; last-position logits."""
        if ids.shape[0] != self.batch:
            raise ValueError(f"prefill batch {ids.shape[0]} != decoder batch {self.batch}")
        self.cache.length = 0
        return forward_cached(self.model, ids, self.cache)

    @torch.no_grad()
    def step(self) -> torch.Tensor:
        """One static-shape decode step for ``self.tok`` at position ``self.pos`` (the body the
        graph records).  Returns logits ``[B, V]``."""
        m = self.model
        bsz = self.batch
        x = m.token_embedding(self.tok) + m.position_embedding(self.pos)[None]  # [B, 1, d]
        hidden = ~(self._slots <= self.pos)  # [cap]: cache slots after this position
        for i, blk in enumerate(m.blocks):
            a = blk.attn
            heads = a.qkv_proj(blk.ln_1(x)).view(bsz, 1, 3, a.n_heads, a.head_dim)
            q, k, v = (t.transpose(1, 2) for t in heads.unbind(dim=2))  # [B, H, 1, hd]
            kc, vc = self.cache.keys[i], self.cache.values[i]
            kc.index_copy_(2, self.pos, k)
            vc.index_copy_(2, self.pos, v)
            s = torch.matmul(q, kc.transpose(-1, -2)) * (a.head_dim**-0.5)  # [B, H, 1, cap]
            s = s.to(torch.promote_types(s.dtype, torch.float32)).masked_fill(hidden, float("-inf"))
            att = torch.matmul(torch.softmax(s, dim=-1).to(vc.dtype), vc)  # [B, H, 1, hd]
            x = x + a.out_proj(att.transpose(1, 2).reshape(bsz, 1, a.d_model))
            x = x + blk.mlp_proj(blk.mlp_act(blk.mlp_fc(blk.ln_2(x))))
        return m.lm_head(m.ln_f(x))[:, -1]

    # -- graph -----------------------------------------------------------------------------

    def _capture(self) -> None:
        # warm-up on a side stream (library handles, allocator pools), then record; the warm-up
        # writes cache slot `pos`, which the next real step overwrites anyway
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for _ in range(2):
                self.step()
        torch.cuda.current_stream(self.device).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            self.logits = self.step()
        self.graph = graph

    @torch.no_grad()
    def decode(self, tokens: torch.Tensor) -> torch.Tensor:
        """Append ``tokens`` ``[B, 1]`` at the next position; logits ``[B, V]`` of that position.

        With a graph the returned tensor is the graph's static output: it is overwritten by the
        next call (clone it to keep it)."""
        if self.cache.length >= self.cache.capacity:
            raise ValueError("KV cache full: context reached block_size")
        self.tok.copy_(tokens)
        self.pos.fill_(self.cache.length)
        if not self.use_graph:
            out = self.step()
        else:
            if self.graph is None:
                self._capture()
            assert self.graph is not None and self.logits is not None
            self.graph.replay()
            out = self.logits
        self.cache.length += 1
        return out
