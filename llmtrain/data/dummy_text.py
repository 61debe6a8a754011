"""``dummy_text``: tiny synthetic copy task (reference ``data/dummy_text.py:15-153``).

Semantics kept exactly (tests and the ``gpt_smoke`` loss-goes-to-zero behaviour depend on them):
``labels == input_ids`` (copy task), ``T = min(block_size, 8)``, per-example generator seeded
``seed + index`` when deterministic, ``min(max_steps * micro_batch, 128)`` train examples and
``min(train // 5, 32)`` validation examples seeded ``seed + 1000``; workers forced to 0.
"""

from __future__ import annotations

from typing import Any

import torch
import torch.distributed as dist
from torch.utils.data import DataLoader, Dataset

from llmtrain.config.schemas import RunConfig
from llmtrain.data._sharding import make_loader
from llmtrain.data.base import DataModule
from llmtrain.registry.data import register_data_module

__all__ = ["DummyTextDataModule"]


class _RandomTokens(Dataset):
    def __init__(self, n: int, seq_len: int, vocab: int, deterministic: bool, seed: int) -> None:
        self.n, self.seq_len, self.vocab = n, seq_len, vocab
        self.deterministic, self.seed = deterministic, seed

    def __len__(self) -> int:
        return self.n

    def __getitem__(self, index: int) -> dict[str, torch.Tensor]:
        gen = None
        if self.deterministic:
            gen = torch.Generator().manual_seed(self.seed + index)
        ids = torch.randint(0, self.vocab, (self.seq_len,), dtype=torch.long, generator=gen)
        return {"input_ids": ids, "labels": ids.clone(), "attention_mask": torch.ones_like(ids)}


@register_data_module("dummy_text")
class DummyTextDataModule(DataModule):
    def __init__(self) -> None:
        self._cfg: RunConfig | None = None
        self._train: Dataset | None = None
        self._val: Dataset | None = None

    def setup(self, cfg: RunConfig, tokenizer: Any | None = None) -> None:
        self._cfg = cfg
        vocab = cfg.model.vocab_size or 128
        seq_len = max(1, min(cfg.model.block_size, 8))
        n_train = max(1, min(cfg.trainer.max_steps * cfg.trainer.micro_batch_size, 128))
        n_val = max(1, min(n_train // 5, 32))
        det, seed = cfg.run.deterministic, cfg.run.seed
        self._train = _RandomTokens(n_train, seq_len, vocab, det, seed)
        self._val = _RandomTokens(n_val, seq_len, vocab, det, seed + 1000)

    def train_dataloader(self) -> DataLoader:
        if self._cfg is None or self._train is None:
            raise RuntimeError("setup must be called before train_dataloader")
        return make_loader(self._train, self._cfg, train=True, num_workers=0, dist_api=dist)

    def val_dataloader(self) -> DataLoader | None:
        if self._cfg is None:
            raise RuntimeError("setup must be called before val_dataloader")
        if self._val is None:
            return None
        return make_loader(self._val, self._cfg, train=False, num_workers=0, dist_api=dist)
