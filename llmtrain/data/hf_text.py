"""``hf_text``: Hugging Face text dataset → tokenized ``block_size + 1`` windows.

Reference ``data/hf_text.py:16-240``: ``datasets.load_dataset(name, config, split, cache_dir)``;
rows tokenized with ``tokenizer.encode``; token ids concatenated per ``Dataset.map`` batch and
cut into ``block_size + 1`` chunks (``input_ids = chunk[:-1]``, ``labels = chunk[1:]``, mask all
ones; the tail of each map batch is dropped — SURVEY Q16); processed splits cached at
``{cache_dir}/processed/{name}__{config}__b{block}__{split}``.  ``datasets`` is imported lazily.
"""

from __future__ import annotations

from pathlib import Path
from typing import Any

import torch
import torch.distributed as dist
from torch.utils.data import DataLoader

from llmtrain.config.schemas import RunConfig
from llmtrain.data._sharding import make_loader
from llmtrain.data.base import DataModule
from llmtrain.registry.data import register_data_module

__all__ = ["HFTextDataModule"]


def _collate(rows: list[dict[str, list[int]]]) -> dict[str, torch.Tensor]:
    return {
        key: torch.tensor([row[key] for row in rows], dtype=torch.long)
        for key in ("input_ids", "labels", "attention_mask")
    }


def _chunker(block_size: int):
    width = block_size + 1

    def chunk(batch: dict[str, list[list[int]]]) -> dict[str, list[list[int]]]:
        stream = [tok for ids in batch["token_ids"] for tok in ids]
        usable = len(stream) - len(stream) % width
        windows = [stream[i : i + width] for i in range(0, usable, width)]
        return {
            "input_ids": [w[:-1] for w in windows],
            "labels": [w[1:] for w in windows],
            "attention_mask": [[1] * block_size for _ in windows],
        }

    return chunk


@register_data_module("hf_text")
class HFTextDataModule(DataModule):
    def __init__(self) -> None:
        self._cfg: RunConfig | None = None
        self._train_dataset: Any | None = None
        self._val_dataset: Any | None = None

    _collate_batch = staticmethod(_collate)

    def setup(self, cfg: RunConfig, tokenizer: Any | None = None) -> None:
        if cfg.data.dataset_name is None:
            raise ValueError("hf_text requires data.dataset_name to be configured.")
        if cfg.data.text_column is None:
            raise ValueError("hf_text requires data.text_column to be configured.")
        if tokenizer is None:
            raise ValueError("hf_text requires a tokenizer instance.")
        if not hasattr(tokenizer, "encode"):
            raise ValueError("hf_text tokenizer must provide an encode(text) method.")
        from datasets import load_dataset, load_from_disk  # type: ignore[import-untyped]

        self._cfg = cfg
        prepare = lambda split: self._prepare_split(  # noqa: E731
            split=split, cfg=cfg, tokenizer=tokenizer, text_column=cfg.data.text_column,
            load_dataset=load_dataset, load_from_disk=load_from_disk,
        )
        self._train_dataset = prepare(cfg.data.train_split)
        self._val_dataset = prepare(cfg.data.val_split)

    def _processed_cache_path(self, cfg: RunConfig, split: str) -> Path:
        name = (cfg.data.dataset_name or "unknown").replace("/", "__")
        config = (cfg.data.dataset_config or "default").replace("/", "__")
        return Path(cfg.data.cache_dir) / "processed" / f"{name}__{config}__b{cfg.model.block_size}__{split}"

    def _prepare_split(self, *, split, cfg, tokenizer, text_column, load_dataset, load_from_disk):  # type: ignore[no-untyped-def]
        cache = self._processed_cache_path(cfg, split)
        if cache.exists():
            return load_from_disk(str(cache))
        raw = load_dataset(cfg.data.dataset_name, cfg.data.dataset_config, split=split, cache_dir=cfg.data.cache_dir)
        processed = self._tokenize_and_chunk(
            raw_dataset=raw, tokenizer=tokenizer, text_column=text_column, block_size=cfg.model.block_size
        )
        cache.parent.mkdir(parents=True, exist_ok=True)
        processed.save_to_disk(str(cache))
        return processed

    def _tokenize_and_chunk(self, *, raw_dataset, tokenizer, text_column, block_size):  # type: ignore[no-untyped-def]
        def encode(batch: dict[str, list[Any]]) -> dict[str, list[list[int]]]:
            out: list[list[int]] = []
            for text in batch[text_column]:
                if text is None:
                    out.append([])
                    continue
                ids = tokenizer.encode(str(text))
                if not isinstance(ids, list):
                    raise ValueError("Tokenizer encode output must be a list of token ids.")
                out.append([int(t) for t in ids])
            return {"token_ids": out}

        tokenized = raw_dataset.map(
            encode, batched=True, remove_columns=raw_dataset.column_names, desc="Tokenizing"
        )
        return tokenized.map(_chunker(block_size), batched=True, remove_columns=["token_ids"], desc="Chunking")

    def train_dataloader(self) -> DataLoader:
        if self._cfg is None or self._train_dataset is None:
            raise RuntimeError("setup must be called before train_dataloader")
        return make_loader(
            self._train_dataset, self._cfg, train=True, num_workers=self._cfg.data.num_workers, collate_fn=_collate,
            dist_api=dist,
        )

    def val_dataloader(self) -> DataLoader | None:
        if self._cfg is None:
            raise RuntimeError("setup must be called before val_dataloader")
        if self._val_dataset is None:
            return None
        return make_loader(
            self._val_dataset, self._cfg, train=False, num_workers=self._cfg.data.num_workers, collate_fn=_collate,
            dist_api=dist,
        )
