"""GPT-2 tokenizer resolution.

The reference hard-requires ``tiktoken`` (``models/gpt.py:210-212``).  This build prefers it
when importable and otherwise falls back to :class:`ByteLevelTokenizer` — a dependency-free,
deterministic byte tokenizer that lives in the GPT-2 id space (``n_vocab = 50257``; ids 0-255
are raw UTF-8 bytes).  It keeps every code path that needs *a* tokenizer working offline
(vocab-size resolution, ``hf_text`` with local data, notebooks' sampling helpers) and logs a
warning so nobody mistakes it for BPE.
"""

from __future__ import annotations

import functools
import logging
from typing import Any

__all__ = ["ByteLevelTokenizer", "GPT2_VOCAB_SIZE", "get_gpt2_tokenizer"]

GPT2_VOCAB_SIZE = 50257
logger = logging.getLogger(__name__)


class ByteLevelTokenizer:
    """UTF-8 bytes as token ids, reported in a GPT-2 sized vocabulary."""

    name = "byte-level-fallback"

    def __init__(self, n_vocab: int = GPT2_VOCAB_SIZE) -> None:
        self.n_vocab = n_vocab
        self.eot_token = n_vocab - 1

    def encode(self, text: str, **_: Any) -> list[int]:
        return list(text.encode("utf-8"))

    def decode(self, ids: list[int]) -> str:
        return bytes(i for i in ids if 0 <= i < 256).decode("utf-8", errors="replace")


@functools.lru_cache(maxsize=1)
def get_gpt2_tokenizer() -> Any:
    try:
        import tiktoken  # type: ignore[import-not-found]

        return tiktoken.get_encoding("gpt2")
    except Exception as exc:  # ModuleNotFoundError, or no cached BPE ranks offline
        logger.warning("tiktoken gpt2 encoding unavailable (%s); using ByteLevelTokenizer", exc)
        return ByteLevelTokenizer()
