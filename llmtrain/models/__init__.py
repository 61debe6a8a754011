"""Model adapters (``gpt``, ``dummy_gpt``)."""

from llmtrain.models.base import LazyFloat, ModelAdapter

__all__ = ["LazyFloat", "ModelAdapter"]
