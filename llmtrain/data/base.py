"""``DataModule`` plugin contract (reference ``data/base.py:11-24``).

Batch contract: ``{"input_ids": long[B,T], "labels": long[B,T], "attention_mask": long[B,T]}``
with labels already aligned to the prediction target (the loss never shifts them).
"""

from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any

from torch.utils.data import DataLoader

from llmtrain.config.schemas import RunConfig

__all__ = ["DataModule"]


class DataModule(ABC):
    @abstractmethod
    def setup(self, cfg: RunConfig, tokenizer: Any | None = None) -> None: ...

    @abstractmethod
    def train_dataloader(self) -> DataLoader: ...

    @abstractmethod
    def val_dataloader(self) -> DataLoader | None: ...
