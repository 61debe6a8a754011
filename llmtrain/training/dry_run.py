"""Forward-only sanity run (reference ``training/dry_run.py:15-87``).

Runs ``min(5, max_steps)`` batches under ``no_grad`` and logs the loss and step time.  Unlike
the reference (which always forces CPU) it runs on the configured runtime device.
"""

from __future__ import annotations

import logging
import time
from dataclasses import dataclass

import torch

from llmtrain.config.schemas import RunConfig
from llmtrain.registry import initialize_registries
from llmtrain.registry.data import get_data_module
from llmtrain.registry.models import get_model_adapter
from llmtrain.runtime.device import resolve_policy

__all__ = ["DEFAULT_DRY_RUN_STEPS", "DryRunResult", "run_dry_run"]

DEFAULT_DRY_RUN_STEPS = 5


@dataclass(frozen=True)
class DryRunResult:
    resolved_model_adapter: str
    resolved_data_module: str
    steps_executed: int


def _resolve_dry_run_steps(cfg: RunConfig) -> int:
    return min(max(DEFAULT_DRY_RUN_STEPS, 1), cfg.trainer.max_steps)


def run_dry_run(cfg: RunConfig, *, logger: logging.Logger | None = None) -> DryRunResult:
    log = logger or logging.getLogger(__name__)
    initialize_registries()
    adapter = get_model_adapter(cfg.model.name)()
    data = get_data_module(cfg.data.name)()
    model = adapter.build_model(cfg)
    data.setup(cfg, tokenizer=adapter.build_tokenizer(cfg))
    loader = data.train_dataloader()

    policy = resolve_policy(cfg) if cfg.run.device in ("cpu", "cuda", "rocm") else None
    device = policy.device if policy is not None else torch.device("cpu")
    model = model.to(device).train()
    steps = _resolve_dry_run_steps(cfg)
    executed = 0
    batches = iter(loader)
    with torch.no_grad():
        for step in range(1, steps + 1):
            try:
                batch = next(batches)
            except StopIteration:
                break
            batch = {k: v.to(device) if torch.is_tensor(v) else v for k, v in batch.items()}
            t0 = time.perf_counter()
            loss, metrics = adapter.compute_loss(model, batch)
            value = float(metrics.get("loss", loss))
            elapsed_ms = (time.perf_counter() - t0) * 1000.0
            executed += 1
            log.info("Dry-run step %s/%s loss=%.4f step_time_ms=%.2f", step, steps, value, elapsed_ms)
    return DryRunResult(cfg.model.name, cfg.data.name, executed)
