"""``synthetic_tokens``: full-``block_size`` next-token windows with no tokenizer and no network.

This is the "gpt_wikitext-shaped synthetic tokens" configuration of the benchmark: windows of
exactly ``block_size`` tokens with ``labels = input_ids`` shifted by one (the ``hf_text``
contract, reference ``data/hf_text.py:150-162``) over ``model.vocab_size`` ids.

Token streams come from a seeded sparse Markov chain — every token has ``branching`` possible
successors drawn once from the seed — so the data is *learnable* (entropy ``ln(branching)`` per
token) and validation loss is a meaningful convergence / parity signal, unlike uniform noise.
``data.extra`` knobs: ``train_sequences`` (4096), ``val_sequences`` (256), ``branching`` (4),
``process`` (``"markov"`` or ``"uniform"``).
"""

from __future__ import annotations

from typing import Any

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset

from llmtrain.config.schemas import RunConfig
from llmtrain.data._sharding import make_loader
from llmtrain.data.base import DataModule
from llmtrain.registry.data import register_data_module

__all__ = ["SyntheticTokensDataModule", "markov_streams"]


def markov_streams(
    n_seq: int, length: int, vocab: int, *, branching: int, seed: int, table_seed: int
) -> np.ndarray:
    """``[n_seq, length]`` int64 token streams of a sparse Markov chain (vectorised over streams)."""
    table_rng = np.random.default_rng(table_seed)
    successors = table_rng.integers(0, vocab, size=(vocab, branching), dtype=np.int64)
    rng = np.random.default_rng(seed)
    out = np.empty((n_seq, length), dtype=np.int64)
    out[:, 0] = rng.integers(0, vocab, size=n_seq)
    choices = rng.integers(0, branching, size=(n_seq, length - 1))
    for t in range(1, length):
        out[:, t] = successors[out[:, t - 1], choices[:, t - 1]]
    return out


class _Windows(Dataset):
    def __init__(self, streams: np.ndarray) -> None:
        self.streams = torch.from_numpy(streams)

    def __len__(self) -> int:
        return self.streams.shape[0]

    def __getitem__(self, index: int) -> dict[str, torch.Tensor]:
        row = self.streams[index]
        ids = row[:-1]
        return {"input_ids": ids, "labels": row[1:], "attention_mask": torch.ones_like(ids)}


@register_data_module("synthetic_tokens")
class SyntheticTokensDataModule(DataModule):
    def __init__(self) -> None:
        self._cfg: RunConfig | None = None
        self._train: Dataset | None = None
        self._val: Dataset | None = None

    def setup(self, cfg: RunConfig, tokenizer: Any | None = None) -> None:
        vocab = cfg.model.vocab_size or getattr(tokenizer, "n_vocab", None)
        if not vocab:
            raise ValueError("synthetic_tokens needs model.vocab_size (or a tokenizer with n_vocab)")
        extra = cfg.data.extra
        length = cfg.model.block_size + 1
        branching = int(extra.get("branching", 4))
        process = extra.get("process", "markov")
        seed = cfg.run.seed
        n_train = int(extra.get("train_sequences", 4096))
        n_val = int(extra.get("val_sequences", 256))

        def gen(n: int, stream_seed: int) -> np.ndarray:
            if process == "uniform":
                return np.random.default_rng(stream_seed).integers(0, vocab, size=(n, length), dtype=np.int64)
            if process != "markov":
                raise ValueError(f"unknown synthetic process {process!r}")
            return markov_streams(n, length, vocab, branching=branching, seed=stream_seed, table_seed=seed)

        self._cfg = cfg
        self._train = _Windows(gen(n_train, seed + 1))
        self._val = _Windows(gen(n_val, seed + 2)) if n_val > 0 else None

    def train_dataloader(self) -> DataLoader:
        if self._cfg is None or self._train is None:
            raise RuntimeError("setup must be called before train_dataloader")
        pin = self._cfg.run.device in ("cuda", "rocm")
        return make_loader(self._train, self._cfg, train=True, num_workers=0, pin_memory=pin)

    def val_dataloader(self) -> DataLoader | None:
        if self._cfg is None:
            raise RuntimeError("setup must be called before val_dataloader")
        if self._val is None:
            return None
        pin = self._cfg.run.device in ("cuda", "rocm")
        return make_loader(self._val, self._cfg, train=False, num_workers=0, pin_memory=pin)
