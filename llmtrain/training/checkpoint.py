"""Checkpoints: ``<run_dir>/checkpoints/step_{step:06d}.pt`` (reference ``training/checkpoint.py``).

Payload keys (the 6-key contract): ``step``, ``model_state_dict`` (fp32 master weights, the
``causal_mask`` buffers, tied ``lm_head``/``token_embedding`` aliases), ``optimizer_state_dict``
(``torch.optim.AdamW`` layout), ``scheduler_state_dict`` (LambdaLR), ``rng_states``
(python/numpy/torch[/cuda]) and ``config``.  An optional seventh key ``llmtrain_extra`` carries
resume metadata (world size, data position); readers that do not know it ignore it.

Improvements over the reference: writes are atomic (``.tmp`` + ``os.replace``; a crash never
leaves a truncated "latest" file) and loading always uses the safe ``weights_only=True``
unpickler (never arbitrary code);
the numpy types a reference checkpoint stores in ``rng_states["numpy"]`` are allow-listed
explicitly so reference checkpoints still load.
"""

from __future__ import annotations

import logging
import os
import random
from pathlib import Path
from typing import Any, TypedDict

import numpy as np
import torch

from llmtrain.config.schemas import RunConfig

__all__ = [
    "CheckpointManager",
    "CheckpointPayload",
    "REQUIRED_KEYS",
    "capture_rng_states",
    "restore_rng_states",
]

logger = logging.getLogger(__name__)


class CheckpointPayload(TypedDict):
    step: int
    model_state_dict: dict[str, Any]
    optimizer_state_dict: dict[str, Any]
    scheduler_state_dict: dict[str, Any]
    rng_states: dict[str, Any]
    config: dict[str, Any]


REQUIRED_KEYS = frozenset(CheckpointPayload.__annotations__)


def _step_of(path: Path) -> int:
    return int(path.stem.split("_")[1])


def _numpy_safe_globals() -> list[Any]:
    """numpy objects found in reference checkpoints' ``np.random.get_state()`` tuple."""
    core = getattr(np, "_core", None) or np.core  # numpy 2 renamed numpy.core → numpy._core
    return [core.multiarray._reconstruct, np.ndarray, np.dtype, type(np.dtype(np.uint32))]


def restore_rng_states(states: dict[str, Any]) -> None:
    random.setstate(states["python"])
    name, key, *rest = states["numpy"]
    np.random.set_state((name, np.asarray(key, dtype=np.uint32), *rest))
    torch.random.set_rng_state(states["torch"])
    if "cuda" in states and torch.cuda.is_available():
        cuda_states = states["cuda"][: torch.cuda.device_count()]
        torch.cuda.set_rng_state_all(cuda_states)


def capture_rng_states() -> dict[str, Any]:
    np_state = np.random.get_state()
    states: dict[str, Any] = {
        "python": random.getstate(),
        # numpy's legacy tuple with its key array as a plain list → loadable with weights_only
        "numpy": (np_state[0], np_state[1].tolist(), *np_state[2:]),
        "torch": torch.random.get_rng_state(),
    }
    if torch.cuda.is_available():
        states["cuda"] = torch.cuda.get_rng_state_all()
    return states


class CheckpointManager:
    def __init__(self, checkpoint_dir: Path, keep_last_k: int = 3) -> None:
        self._checkpoint_dir = Path(checkpoint_dir)
        self._keep_last_k = keep_last_k
        self._checkpoint_dir.mkdir(parents=True, exist_ok=True)

    @property
    def directory(self) -> Path:
        return self._checkpoint_dir

    def path_for(self, step: int) -> Path:
        return self._checkpoint_dir / f"step_{step:06d}.pt"

    def save(
        self,
        step: int,
        model: torch.nn.Module,
        optimizer: torch.optim.Optimizer,
        scheduler: Any,
        config: RunConfig,
        *,
        extra: dict[str, Any] | None = None,
    ) -> Path:
        payload: dict[str, Any] = {
            "step": step,
            "model_state_dict": model.state_dict(),
            "optimizer_state_dict": optimizer.state_dict(),
            "scheduler_state_dict": scheduler.state_dict(),
            "rng_states": capture_rng_states(),
            "config": config.model_dump(),
        }
        if extra:
            payload["llmtrain_extra"] = extra
        path = self.path_for(step)
        tmp = path.with_name(path.name + ".tmp")
        torch.save(payload, tmp)
        os.replace(tmp, path)
        logger.info("checkpoint: saved step %d to %s", step, path)
        self._prune_old()
        return path

    def load(self, path: Path, *, map_location: Any = "cpu") -> CheckpointPayload:
        logger.info("checkpoint: loading %s", path)
        with torch.serialization.safe_globals(_numpy_safe_globals()):
            data = torch.load(path, map_location=map_location, weights_only=True)
        missing = REQUIRED_KEYS - set(data)
        if missing:
            raise ValueError(f"Checkpoint at {path} is missing keys: {missing}")
        return data  # type: ignore[return-value]

    def checkpoints(self) -> list[Path]:
        return sorted(self._checkpoint_dir.glob("step_*.pt"), key=_step_of)

    def latest_checkpoint(self) -> Path | None:
        found = self.checkpoints()
        return found[-1] if found else None

    def _prune_old(self) -> None:
        found = self.checkpoints()
        for stale in found[: max(0, len(found) - self._keep_last_k)]:
            stale.unlink(missing_ok=True)
            logger.debug("checkpoint: pruned %s", stale)
