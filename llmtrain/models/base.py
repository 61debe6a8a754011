"""``ModelAdapter`` plugin contract (reference ``models/base.py:12-27``)."""

from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any

import torch
from torch import nn

from llmtrain.config.schemas import RunConfig

__all__ = ["LazyFloat", "ModelAdapter"]


class ModelAdapter(ABC):
    """Builds a model/tokenizer for a config and computes ``(loss, metrics)`` for a batch."""

    @abstractmethod
    def build_model(self, cfg: RunConfig) -> nn.Module: ...

    @abstractmethod
    def build_tokenizer(self, cfg: RunConfig) -> Any | None: ...

    @abstractmethod
    def compute_loss(
        self, model: nn.Module, batch: dict[str, torch.Tensor]
    ) -> tuple[torch.Tensor, dict[str, float]]: ...


class LazyFloat:
    """A metric value backed by a 0-d device tensor, materialised only when read.

    The reference adapters return ``{"loss": float(loss.item())}`` — a host sync on every
    micro-step (``models/gpt.py:271``).  Returning a ``LazyFloat`` keeps the ``dict[str, float]``
    contract for consumers that call ``float()``/``math.isfinite``/formatting on it, while the
    trainer accumulates the underlying tensor on the device and syncs once per log interval.
    """

    __slots__ = ("tensor", "_cached")

    def __init__(self, tensor: torch.Tensor) -> None:
        self.tensor = tensor.detach()
        self._cached: float | None = None

    def __float__(self) -> float:
        if self._cached is None:
            self._cached = float(self.tensor.item())
        return self._cached

    def __format__(self, spec: str) -> str:
        return format(float(self), spec)

    def __repr__(self) -> str:
        return f"LazyFloat({float(self)!r})"

    def __eq__(self, other: object) -> bool:
        try:
            return float(self) == float(other)  # type: ignore[arg-type]
        except (TypeError, ValueError):
            return NotImplemented

    def __lt__(self, other: object) -> bool:
        return float(self) < float(other)  # type: ignore[arg-type]

    def __gt__(self, other: object) -> bool:
        return float(self) > float(other)  # type: ignore[arg-type]

    def __add__(self, other: object) -> float:
        return float(self) + float(other)  # type: ignore[arg-type]

    __radd__ = __add__

    def __hash__(self) -> int:
        return hash(float(self))


def validate_lm_batch(batch: dict[str, torch.Tensor], *, min_len: int = 1) -> None:
    """Shape/dtype checks shared by the LM adapters (reference ``models/gpt.py:221-252``)."""
    input_ids, labels = batch["input_ids"], batch["labels"]
    mask = batch.get("attention_mask")
    if input_ids.dim() != 2 or labels.dim() != 2:
        raise ValueError(
            "Expected input_ids and labels to be 2D (B, T); "
            f"got {tuple(input_ids.shape)} and {tuple(labels.shape)}."
        )
    if input_ids.shape != labels.shape:
        raise ValueError(
            "Expected input_ids and labels to have the same shape; "
            f"got {tuple(input_ids.shape)} vs {tuple(labels.shape)}."
        )
    if input_ids.dtype != torch.long or labels.dtype != torch.long:
        raise ValueError(
            f"Expected input_ids and labels to be torch.long; got {input_ids.dtype} and {labels.dtype}."
        )
    if input_ids.size(1) < min_len:
        raise ValueError("Expected sequence length >= 2 for next-token loss.")
    if mask is None:
        return
    if mask.dim() != 2:
        raise ValueError(f"Expected attention_mask to be 2D (B, T); got {tuple(mask.shape)}.")
    if mask.shape != input_ids.shape:
        raise ValueError(
            "Expected attention_mask to match input_ids shape; "
            f"got {tuple(mask.shape)} vs {tuple(input_ids.shape)}."
        )
    if mask.dtype not in (torch.bool, torch.long, torch.int64):
        raise ValueError(f"Expected attention_mask to be bool or int64; got {mask.dtype}.")
