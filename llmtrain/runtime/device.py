"""Device, precision and seeding policy — decided once per run and passed down.

* ``run.device``: ``cpu`` | ``mps`` | ``cuda``/``rocm`` → ``cuda:<local_rank>`` (HIP GPU).
* ``run.precision``: ``fp32`` (reference numerics) | ``bf16`` (MI355X compute path).
* ``run.seed`` seeds python/numpy/torch (+ all HIP devices) BEFORE the model is built — the
  reference validates but never applies the seed; applying it here is an
  intentional, documented fix so runs are reproducible and ranks initialise identically.
"""

from __future__ import annotations

import random
from dataclasses import dataclass

import numpy as np
import torch

from llmtrain.config.schemas import RunConfig

__all__ = ["RuntimePolicy", "decorrelate_rank_streams", "resolve_policy", "seed_everything", "settle_fused_path"]


@dataclass(frozen=True)
class RuntimePolicy:
    device: torch.device
    compute_dtype: torch.dtype
    use_fused: bool

    @property
    def is_gpu(self) -> bool:
        return self.device.type == "cuda"

    def autocast(self):  # type: ignore[no-untyped-def]
        """Autocast context for the module path (no-op for fp32 or the fused engine)."""
        import contextlib

        if self.is_gpu and self.compute_dtype == torch.bfloat16 and not self.use_fused:
            return torch.autocast(device_type="cuda", dtype=torch.bfloat16)
        return contextlib.nullcontext()


def _device_for(cfg: RunConfig, local_rank: int) -> torch.device:
    if cfg.run.device in ("cuda", "rocm"):
        if not torch.cuda.is_available():
            raise RuntimeError("run.device requests a GPU but no HIP device is visible")
        return torch.device("cuda", local_rank % max(1, torch.cuda.device_count()))
    return torch.device(cfg.run.device)


def resolve_policy(cfg: RunConfig, *, local_rank: int = 0, fused_capable: bool = False) -> RuntimePolicy:
    device = _device_for(cfg, local_rank)
    compute = torch.bfloat16 if cfg.run.precision == "bf16" else torch.float32
    setting = cfg.model.extra.get("fused", "auto")
    if setting == "auto":
        use_fused = fused_capable and device.type == "cuda" and compute == torch.bfloat16
    else:
        use_fused = bool(setting) and fused_capable
    return RuntimePolicy(device=device, compute_dtype=compute, use_fused=use_fused)


def seed_everything(seed: int) -> None:
    random.seed(seed)
    np.random.seed(seed % 2**32)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def decorrelate_rank_streams(rank: int) -> int:
    """Give each data-parallel rank its own torch RNG stream from here on.

    Called AFTER the model is built (parameter init stays identical on every rank) and again after
    a resume restored rank 0's checkpointed RNG state onto every rank.  Every rank draws the same
    value from the (identical) generator state and reseeds with that value mixed with its rank, so
    dropout masks — the fused engine's per-forward site seed and the module path's ``nn.Dropout``
    on CPU or GPU — differ across ranks like the reference's unseeded per-process generators, yet a
    run stays reproducible.  Returns the new seed."""
    draw = int(torch.randint(0, 2**62, (1,)).item())
    seed = (draw ^ ((rank + 1) * 0x9E3779B97F4A7C15)) % (2**63 - 1)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    return seed


def settle_fused_path(policy: RuntimePolicy, cfg: RunConfig, supported: bool) -> RuntimePolicy:
    """The fused engine was chosen but does not cover this model shape on ``policy.device``.

    On the GPU the module path (torch SDPA + autograd + torch AdamW) is not a production backend:
    an uncovered shape is an error unless the config opts in with
    ``model.extra.allow_module_fallback: true`` (or asks for the module path with
    ``model.extra.fused: false``).  On CPU the module path is the reference numerics and is taken
    silently.
    """
    if not policy.use_fused or supported:
        return policy
    if policy.device.type == "cuda" and not cfg.model.extra.get("allow_module_fallback", False):
        raise ValueError(
            f"the fused MI355X engine does not cover this model shape (d_model={cfg.model.d_model}, "
            f"n_heads={cfg.model.n_heads}, d_ff={cfg.model.d_ff}: head dims must be multiples of 8 up to 64, "
            "or 128; d_model % 4 == 0 and <= 2048; d_ff % 8 == 0); set model.extra.allow_module_fallback: true "
            "to train on the plain PyTorch module path instead, or model.extra.fused: false"
        )
    return RuntimePolicy(device=policy.device, compute_dtype=policy.compute_dtype, use_fused=False)
