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
from pathlib import Path

import torch
import torch.distributed as dist

from llmtrain.config.schemas import RunConfig
from llmtrain.parallel import comm

__all__ = ["DDPState", "ReplicaMismatchError", "resolve_backend", "setup_ddp", "teardown_ddp", "verify_replicas"]

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
    if backend == "nccl":
        comm.configure_rccl_env(cfg.ddp.extra, rank, default_dir=Path(cfg.output.root_dir) / "rccl")
    probe_device = torch.device("cpu")
    if _uses_gpu(cfg) and torch.cuda.is_available():
        # local_rank modulo the visible devices, as runtime/device.py picks the device: identity on a
        # full node; on a box with fewer GPUs than ranks (a gloo rehearsal of the multi-rank path)
        # ranks share devices — RCCL itself refuses two ranks on one device
        dev = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev)
        probe_device = torch.device("cuda", dev)
        if backend == "nccl":
            kwargs["device_id"] = torch.device("cuda", dev)
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
    # startup transport check: bus bandwidth of a few large all-reduces + RCCL's transport lines
    comm.check_transport(probe_device, cfg.ddp.extra, rank=rank)
    return state


def teardown_ddp() -> None:
    comm.relay_warnings()
    if dist.is_initialized():
        logger.info("Destroying DDP process group")
        dist.destroy_process_group()


class ReplicaMismatchError(RuntimeError):
    """Data-parallel ranks hold different parameters (SURVEY §5.2 consistency check)."""


def verify_replicas(params, *, device, tag: str, rtol: float = 0.0) -> tuple[float, float]:  # type: ignore[no-untyped-def]
    """Compare a parameter checksum across ranks: ``(Σ p, Σ p²)`` in fp64 on every rank,
    all-reduced with MAX and MIN (two tiny collectives).  Raises :class:`ReplicaMismatchError` when
    any rank differs by more than ``rtol`` (0 = bitwise-equal sums, which identical replicas always
    produce because every rank reduces the same values in the same order).  Called after the
    data-parallel wrap (rank-0 broadcast) and after a resume."""
    import torch

    parts = []
    with torch.no_grad():
        for p in params:
            v = p.detach().to(torch.float64)
            parts.append(torch.stack([v.sum(), (v * v).sum()]))
    total = torch.stack(parts).sum(dim=0).to(device) if parts else torch.zeros(2, dtype=torch.float64, device=device)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(total[0]), float(total[1])
    hi, lo = total.clone(), total.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    spread = (hi - lo).abs()
    limit = rtol * hi.abs().clamp_min(1.0)
    if bool((spread > limit).any()):
        raise ReplicaMismatchError(
            f"{tag}: parameter checksums differ across ranks (sum spread {float(spread[0]):.3e}, "
            f"sumsq spread {float(spread[1]):.3e})"
        )
    return float(total[0]), float(total[1])
