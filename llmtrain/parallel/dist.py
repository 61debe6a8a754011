"""Process-group bootstrap for data parallelism (reference ``distributed/__init__.py:19-153``).

Rank / world size / local rank come from the environment (``torchrun``, the K8s entrypoint)
and fall back to the ``ddp.*`` config fields.  On a GPU run the device is bound BEFORE the
process group is created (``torch.cuda.set_device(local_rank)``; the reference never binds a
device) and the backend is RCCL — torch's ``"nccl"`` backend name on ROCm — which runs its
rings over the xGMI links between the MI355X GPUs of a node.
"""

from __future__ import annotations

import logging
import os
from dataclasses import dataclass
from datetime import timedelta

import torch
import torch.distributed as dist

from llmtrain.config.schemas import RunConfig

__all__ = ["DDPState", "resolve_backend", "setup_ddp", "teardown_ddp"]

logger = logging.getLogger(__name__)


@dataclass(frozen=True)
class DDPState:
    rank: int
    world_size: int
    local_rank: int
    is_main: bool

    def __post_init__(self) -> None:
        if self.is_main != (self.rank == 0):
            raise ValueError("is_main must be True when rank == 0 and False otherwise")


def _env_int(name: str) -> int | None:
    raw = os.environ.get(name)
    if raw is None:
        return None
    try:
        return int(raw)
    except ValueError:
        raise RuntimeError(f"Env var {name} must be an integer, got: {raw!r}") from None


def _resolve_int(env_name: str, fallback: int | None, label: str) -> int:
    value = _env_int(env_name)
    if value is None:
        value = fallback
    if value is None:
        field = label.rsplit(".", 1)[-1]
        raise RuntimeError(f"DDP {field} not found in env ({env_name}) or config ({label})")
    return value


def resolve_backend(cfg: RunConfig) -> str:
    """``rccl`` is an alias of torch's ``nccl`` backend (RCCL on ROCm)."""
    backend = cfg.ddp.backend
    return "nccl" if backend in ("nccl", "rccl") else backend


def _uses_gpu(cfg: RunConfig) -> bool:
    return cfg.run.device in ("cuda", "rocm")


def setup_ddp(cfg: RunConfig) -> DDPState:
    if dist.is_initialized():
        rank, world = dist.get_rank(), dist.get_world_size()
        local = _env_int("LOCAL_RANK")
        if local is None:
            local = cfg.ddp.local_rank if cfg.ddp.local_rank is not None else rank
        state = DDPState(rank=rank, world_size=world, local_rank=local, is_main=rank == 0)
        logger.warning("DDP process group already initialised — returning existing state: %s", state)
        return state

    under_launcher = os.environ.get("RANK") is not None
    rank = _resolve_int("RANK", cfg.ddp.rank, "ddp.rank")
    world = _resolve_int("WORLD_SIZE", cfg.ddp.world_size, "ddp.world_size")
    local = _resolve_int("LOCAL_RANK", cfg.ddp.local_rank, "ddp.local_rank")
    if not under_launcher:
        if cfg.ddp.master_addr is not None:
            os.environ.setdefault("MASTER_ADDR", cfg.ddp.master_addr)
        if cfg.ddp.master_port is not None:
            os.environ.setdefault("MASTER_PORT", str(cfg.ddp.master_port))

    backend = resolve_backend(cfg)
    kwargs = {}
    if _uses_gpu(cfg) and torch.cuda.is_available():
        torch.cuda.set_device(local)
        if backend == "nccl":
            kwargs["device_id"] = torch.device("cuda", local)
    logger.info(
        "Initialising DDP process group: rank=%d, world_size=%d, local_rank=%d, backend=%s, "
        "init_method=env://",
        rank, world, local, backend,
    )
    dist.init_process_group(
        backend=backend,
        init_method="env://",
        rank=rank,
        world_size=world,
        timeout=timedelta(seconds=cfg.ddp.timeout_sec),
        **kwargs,
    )
    state = DDPState(rank=rank, world_size=world, local_rank=local, is_main=rank == 0)
    logger.info("DDP process group initialised: %s", state)
    return state


def teardown_ddp() -> None:
    if dist.is_initialized():
        logger.info("Destroying DDP process group")
        dist.destroy_process_group()
