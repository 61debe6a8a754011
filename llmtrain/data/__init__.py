"""Data modules (``dummy_text``, ``hf_text``, ``synthetic_tokens``)."""

from llmtrain.data.base import DataModule

__all__ = ["DataModule"]
