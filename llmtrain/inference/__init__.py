"""Inference: KV-cached autoregressive sampling for the ``gpt`` model."""

from llmtrain.inference.generate import (
    KVCache,
    forward_cached,
    generate,
    generate_text,
    sample_next_token,
    top_next_tokens,
)
from llmtrain.inference.graph_decode import GraphDecoder

__all__ = ["GraphDecoder", "KVCache", "forward_cached", "generate", "generate_text", "sample_next_token", "top_next_tokens"]
