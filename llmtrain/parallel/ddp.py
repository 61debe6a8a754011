"""Choosing the data-parallel wrapper for a model.

* fused-engine models → :class:`~llmtrain.parallel.reducer.FlatDataParallel` (zero-copy
  bucketed all-reduce driven by the hand-written backward);
* everything else (``dummy_gpt``, module-path ``gpt``) → torch ``DistributedDataParallel`` with
  the constant buffers NOT re-broadcast every forward (``broadcast_buffers=False``)
  and gradients used as bucket views (no extra copy).
"""

from __future__ import annotations

from typing import Any

import torch
from torch import nn
from torch.nn.parallel import DistributedDataParallel

from llmtrain.config.schemas import RunConfig
from llmtrain.parallel.reducer import FlatDataParallel

__all__ = ["unwrap", "wrap_data_parallel"]


def wrap_data_parallel(model: nn.Module, cfg: RunConfig, device: torch.device) -> nn.Module:
    extra = cfg.trainer.extra
    cap_mb = float(extra.get("bucket_cap_mb", 64.0))
    if getattr(model, "engine", None) is not None:
        reduce_dtype = {"bf16": torch.bfloat16, "fp32": None, None: None}[extra.get("grad_reduce_dtype")]
        return FlatDataParallel(model, bucket_cap_mb=cap_mb, reduce_dtype=reduce_dtype)
    kwargs: dict[str, Any] = dict(
        find_unused_parameters=cfg.ddp.find_unused_parameters,
        broadcast_buffers=False,
        gradient_as_bucket_view=True,
        bucket_cap_mb=cap_mb,
    )
    if device.type == "cuda":
        kwargs["device_ids"] = [device.index if device.index is not None else torch.cuda.current_device()]
    return DistributedDataParallel(model, **kwargs)


def unwrap(model: nn.Module) -> nn.Module:
    return getattr(model, "module", model) if isinstance(model, (DistributedDataParallel, FlatDataParallel)) else model
