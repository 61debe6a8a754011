"""Optimizers: torch-layout-compatible fused AdamW over the flat parameter store.

Reference: ``torch.optim.AdamW(model.parameters(), lr, weight_decay)`` with default betas/eps,
decay applied to every parameter (``training/trainer.py:93-97``), and
``clip_grad_norm_`` before each step (``trainer.py:390-393``).

:class:`FusedAdamW` keeps exactly the ``torch.optim.AdamW`` ``state_dict`` layout (a distinct
per-parameter ``step`` fp32 scalar, ``exp_avg``, ``exp_avg_sq``; same ``param_groups`` keys) so checkpoints
move between this build and the reference in both directions, but the update itself is ONE
HIP kernel over the flat buffers: it reads the fp32 master weight, gradient and both moments,
applies the (device-side) gradient-clipping coefficient, writes the new master weight, both
moments AND the bf16 shadow copy used by the next forward — one HBM pass, no per-tensor
launches, no host sync.

Non-finite gradients: :func:`fused_clip_coef` turns a NaN/Inf global norm into a
NaN clip coefficient, and the AdamW kernel then skips the whole update on device — master
weights, both moments and the shadow keep the last good step — and bumps the int32 counters
:attr:`FusedAdamW.skipped` ``[total, consecutive]``.  The Trainer reads them at its log / save
cadence (already host-sync points).  A skipped step still advances the step counter and the LR
schedule (the host cannot know without a sync), so a resumed run replays it identically.
"""

from __future__ import annotations

from collections.abc import Iterable
from typing import Any

import torch
from torch import nn

from llmtrain import ops

__all__ = ["FusedAdamW", "build_optimizer", "fused_clip_coef"]


class FusedAdamW(torch.optim.Optimizer):
    def __init__(
        self,
        params: Iterable[nn.Parameter],
        *,
        store: Any,
        lr: float = 1e-3,
        betas: tuple[float, float] = (0.9, 0.999),
        eps: float = 1e-8,
        weight_decay: float = 1e-2,
    ) -> None:
        defaults = dict(
            lr=lr,
            betas=betas,
            eps=eps,
            weight_decay=weight_decay,
            amsgrad=False,
            maximize=False,
            foreach=None,
            capturable=False,
            differentiable=False,
            fused=None,
            decoupled_weight_decay=True,
        )
        super().__init__(params, defaults)
        if len(self.param_groups) != 1:
            raise ValueError("FusedAdamW supports exactly one parameter group")
        plist = self.param_groups[0]["params"]
        if len(plist) != len(store.params) or not all(store.owns(p) for p in plist):
            raise ValueError("FusedAdamW parameters must be exactly the flat store's parameters")
        self.store = store
        self.exp_avg = torch.zeros_like(store.master)
        self.exp_avg_sq = torch.zeros_like(store.master)
        self._step_count_host = 0
        self._step_tensor = torch.zeros((), dtype=torch.float32)
        self._dyn: torch.Tensor | None = None  # device per-step scalars of a graph-captured step
        # device int32 [total, consecutive] steps skipped for a non-finite gradient norm
        self.skipped = torch.zeros(2, dtype=torch.int32, device=store.master.device)

    # -- torch-compatible state -----------------------------------------------------------

    def _views(self, p: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        off = self.store.offset_of(p)
        n = p.numel()
        return self.exp_avg[off : off + n].view_as(p), self.exp_avg_sq[off : off + n].view_as(p)

    def _materialize_state(self) -> None:
        for p in self.param_groups[0]["params"]:
            st = self.state[p]
            if "exp_avg" not in st or st["exp_avg"].data_ptr() != self._views(p)[0].data_ptr():
                m, v = self._views(p)
                st["step"] = self._step_tensor
                st["exp_avg"] = m
                st["exp_avg_sq"] = v

    def state_dict(self) -> dict[str, Any]:
        """torch.optim.AdamW layout with a DISTINCT fp32 ``step`` tensor per parameter.

        Internally every parameter shares one step counter (the update is one kernel over the
        flat buffers).  Exporting that shared tensor would survive ``torch.save`` as an alias, and
        ``torch.optim.AdamW`` (non-capturable) increments ``state["step"]`` in place once per
        parameter — a shared counter would then advance by #params per step and corrupt the bias
        correction after a resume on the module path or in the reference trainer
        (reference ``training/checkpoint.py:53-68``, ``trainer.py:93-97``)."""
        sd = super().state_dict()
        sd["state"] = {
            k: {**st, "step": st["step"].detach().clone()} if "step" in st else dict(st)
            for k, st in sd["state"].items()
        }
        return sd

    def load_state_dict(self, state_dict: dict[str, Any]) -> None:
        super().load_state_dict(state_dict)
        steps = []
        for p in self.param_groups[0]["params"]:
            st = self.state.get(p)
            if not st:
                continue
            m, v = self._views(p)
            m.copy_(st["exp_avg"].reshape(m.shape))
            v.copy_(st["exp_avg_sq"].reshape(v.shape))
            steps.append(int(float(st["step"])))
        self._step_count_host = max(steps) if steps else 0
        self._step_tensor = torch.tensor(float(self._step_count_host), dtype=torch.float32)
        if steps:
            self._materialize_state()

    def zero_grad(self, set_to_none: bool = True) -> None:  # noqa: ARG002 - grads are views
        self.store.zero_grad()

    # -- update ---------------------------------------------------------------------------

    @torch.no_grad()
    def step(self, closure=None, *, grad_scale: torch.Tensor | None = None):  # type: ignore[override]
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._materialize_state()
        group = self.param_groups[0]
        beta1, beta2 = group["betas"]
        self._step_count_host += 1
        self._step_tensor.fill_(float(self._step_count_host))
        ops.adamw_flat(
            self.store.master,
            self.store.grad,
            self.exp_avg,
            self.exp_avg_sq,
            self.store.shadow,
            lr=float(group["lr"]),
            beta1=float(beta1),
            beta2=float(beta2),
            eps=float(group["eps"]),
            weight_decay=float(group["weight_decay"]),
            step=self._step_count_host,
            grad_scale=grad_scale,
            skipped=self.skipped,
        )
        self.store.mark_shadow_synced()
        return loss


    @property
    def steps_taken(self) -> int:
        """Optimizer steps applied so far (host counter; every parameter's ``step`` in state_dict)."""
        return self._step_count_host

    # -- hipGraph-captured steps (Trainer with trainer.extra.cuda_graph) --------------------

    def stage_graph_step(self) -> None:
        """Host half of a graph-replayed step: advance the step counter and stage this step's
        ``{decay, step_size, bc2_sqrt}`` (from the CURRENT lr, i.e. after the scheduler) into the
        device buffer the captured AdamW kernel reads — the same values :meth:`step` would bake in."""
        self._materialize_state()
        group = self.param_groups[0]
        beta1, beta2 = group["betas"]
        self._step_count_host += 1
        self._step_tensor.fill_(float(self._step_count_host))
        host = torch.ops.llmtrain_hip.adamw_stage_scalars(
            float(group["lr"]), float(beta1), float(beta2), float(group["eps"]), float(group["weight_decay"]),
            self._step_count_host,
        )
        if self._dyn is None:
            self._dyn = torch.empty(3, dtype=torch.float32, device=self.store.master.device)
        self._dyn.copy_(host)

    @torch.no_grad()
    def step_captured(self, *, grad_scale: torch.Tensor | None = None) -> None:
        """Device half, recorded into the graph: the AdamW kernel reading the staged scalars (no host
        state changes, so a capture followed by replays counts each replay exactly once)."""
        if self._dyn is None:
            raise RuntimeError("stage_graph_step() must run before the captured step")
        group = self.param_groups[0]
        beta1, beta2 = group["betas"]
        ops.adamw_flat(
            self.store.master, self.store.grad, self.exp_avg, self.exp_avg_sq, self.store.shadow,
            lr=float(group["lr"]), beta1=float(beta1), beta2=float(beta2), eps=float(group["eps"]),
            weight_decay=float(group["weight_decay"]), step=max(1, self._step_count_host), grad_scale=grad_scale,
            dyn=self._dyn, skipped=self.skipped,
        )
        self.store.mark_shadow_synced()


def fused_clip_coef(
    store: Any, max_norm: float, *, sumsq: torch.Tensor | None = None
) -> tuple[torch.Tensor, torch.Tensor]:
    """Global grad L2 norm and ``min(1, max_norm / (norm + 1e-6))``, both as device scalars (one
    HIP launch after the squared-norm reduction); the coefficient is NaN when the norm is NaN/Inf,
    which makes the fused AdamW skip the step.  ``sumsq``: the squared norm already summed elsewhere
    (the data-parallel reducer's per-bucket partials, :meth:`FlatDataParallel.grad_sumsq`) instead of
    a pass over ``store.grad``."""
    out = ops.clip_coef(ops.sumsq(store.grad) if sumsq is None else sumsq, max_norm)
    return out[0], out[1]


def build_optimizer(model: nn.Module, lr: float, weight_decay: float) -> torch.optim.Optimizer:
    store = getattr(model, "flat_store", None)
    if store is not None:
        return FusedAdamW(model.parameters(), store=store, lr=lr, weight_decay=weight_decay)
    return torch.optim.AdamW(model.parameters(), lr=lr, weight_decay=weight_decay)
