"""Rank sharding shared by the data modules.

A ``DistributedSampler`` is used when a process group with world > 1 is initialised, or —
without one — when the config hints ``ddp.world_size > 1`` (reference ``data/dummy_text.py:95-113``,
``data/hf_text.py:181-198``).  Train shuffles unless ``run.deterministic``; validation never does.
"""

from __future__ import annotations

from typing import Any

import torch.distributed as dist
from torch.utils.data import DataLoader, Dataset
from torch.utils.data.distributed import DistributedSampler

from llmtrain.config.schemas import RunConfig


def world_and_rank(cfg: RunConfig, dist_api: Any = dist) -> tuple[int, int, bool]:
    """``dist_api`` is the ``torch.distributed`` module as the calling data module sees it (each
    module imports it as ``dist`` and passes it, so tests can patch one module's view)."""
    if dist_api.is_available() and dist_api.is_initialized():
        world, rank = dist_api.get_world_size(), dist_api.get_rank()
        return world, rank, world > 1
    world = cfg.ddp.world_size or 1
    rank = cfg.ddp.rank or 0
    return world, rank, world > 1


def make_loader(
    dataset: Dataset,
    cfg: RunConfig,
    *,
    train: bool,
    num_workers: int,
    collate_fn: Any = None,
    pin_memory: bool = False,
    dist_api: Any = dist,
) -> DataLoader:
    world, rank, sharded = world_and_rank(cfg, dist_api)
    shuffle = train and not cfg.run.deterministic
    sampler = None
    if sharded:
        sampler = DistributedSampler(
            dataset, num_replicas=world, rank=rank, shuffle=shuffle, seed=cfg.run.seed
        )
    return DataLoader(
        dataset,
        batch_size=cfg.trainer.micro_batch_size or 1,
        num_workers=num_workers,
        shuffle=sampler is None and shuffle,
        sampler=sampler,
        collate_fn=collate_fn,
        pin_memory=pin_memory,
    )
