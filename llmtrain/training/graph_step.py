"""hipGraph-captured optimizer steps for launch-bound configurations (``trainer.extra.cuda_graph``).

The reference's presets are small models (d_model 64-384, a few thousand tokens per step): on an
MI355X each of their several hundred kernels finishes in a few microseconds, so the eager step is
bound by the host issuing launches, not by the GPU.  This captures ONE whole optimizer step —
gradient zeroing, every micro-batch's fused forward + backward (both HIP streams: the side
stream's weight-gradient GEMMs fork from and join back into the capture stream through the
engine's events), the device-side clip coefficient and the fused AdamW update — into a hipGraph
and replays it for every later step; the host then only copies the next batch into the graph's
static input buffers, stages the step's AdamW scalars (:meth:`FusedAdamW.stage_graph_step`: the
learning rate changes every step and must not be baked in) and launches the graph.

Dropout: the captured kernels keep their site seeds; every dropout kernel also adds a device
word to its seed at entry (``set_dropout_seed_offset``), which the host restages before each
step.  In this mode the per-forward base seed is the micro-batch index and the word is a hash of
(run seed, optimizer step), for eager and replayed steps alike — fresh masks every step, and a
resumed run replays the same masks (no dependence on how many RNG draws happened before).

Scope (checked when the trainer is built, :func:`check_graphable`): the fused engine on a GPU,
the fused AdamW, one process (RCCL collectives are not captured), and batches of one fixed
shape without padding.  A batch that does not fit the captured shape or carries a padding mask
runs eagerly instead (same results, just launch-bound), so correctness never depends on the data.  The first ``warmup`` steps run
eagerly on the capture stream (library handles, workspaces and caches are created outside the
capture), then the step is captured and replayed.
"""

from __future__ import annotations

import logging
from collections.abc import Callable
from typing import Any

import torch

__all__ = ["GraphedStep", "check_graphable"]

logger = logging.getLogger(__name__)


def check_graphable(*, device: torch.device, fused: bool, optimizer: Any, ddp_active: bool) -> None:
    """Raise ``ValueError`` naming the first requirement of a captured step that is not met."""
    from llmtrain.training.optim import FusedAdamW

    if device.type != "cuda":
        raise ValueError("trainer.extra.cuda_graph needs a GPU device")
    if not fused:
        raise ValueError("trainer.extra.cuda_graph needs the fused engine (model.extra.fused)")
    if not isinstance(optimizer, FusedAdamW):
        raise ValueError("trainer.extra.cuda_graph needs the fused AdamW")
    if ddp_active:
        raise ValueError("trainer.extra.cuda_graph is single-process (RCCL collectives are not captured)")


class GraphedStep:
    """Runs optimizer steps: eager for the first ``warmup`` calls, then one captured hipGraph.

    ``eager(batches_on_device)`` runs a whole optimizer step the normal way and returns
    ``(loss, grad_norm)``; ``body(static_batches)`` is the same step written for capture (it must
    not change host-side optimizer state: see :meth:`FusedAdamW.step_captured`); ``after()``
    runs once per step on the host after the step (the LR scheduler)."""

    def __init__(
        self,
        *,
        device: torch.device,
        optimizer: Any,
        eager: Callable[[list[dict[str, Any]]], tuple[torch.Tensor, torch.Tensor]],
        body: Callable[[list[dict[str, Any]]], tuple[torch.Tensor, torch.Tensor]],
        after: Callable[[], None],
        warmup: int = 2,
        engine: Any = None,
        dropout: bool = False,
        run_seed: int = 0,
    ) -> None:
        self._device = device
        self._opt = optimizer
        self._eager = eager
        self._body = body
        self._after = after
        self._warmup = max(1, int(warmup))
        self._calls = 0
        self._stream = torch.cuda.Stream(device=device)
        self._graph: torch.cuda.CUDAGraph | None = None
        self._static: list[dict[str, Any]] | None = None
        self._out: tuple[torch.Tensor, torch.Tensor] | None = None
        self.replays = 0
        self.eager_steps = 0
        self._run_seed = int(run_seed) & 0xFFFFFFFF
        self._seed_word: torch.Tensor | None = None
        self._micro = 0
        if dropout:
            if engine is None:
                raise ValueError("graph-captured dropout needs the fused engine")
            self._seed_word = torch.zeros(1, dtype=torch.int32, device=device)
            engine.drop_seed_source = self._next_base

    # -- dropout seeds -----------------------------------------------------------------------

    def _next_base(self) -> int:
        """Base seed of the next forward in this step: its micro-batch index (captured once)."""
        base = 0x5EED0000 + self._micro
        self._micro += 1
        return base

    def _stage_dropout(self, step_no: int) -> None:
        if self._seed_word is None:
            return
        from llmtrain.ops.reference import mix32_int

        word = mix32_int(self._run_seed ^ ((step_no * 0x9E3779B9) & 0xFFFFFFFF))
        word = word - (1 << 32) if word >= (1 << 31) else word  # int32 view of the uint32
        self._micro = 0
        self._seed_word.fill_(word)

    def _kernels_read_word(self, on: bool) -> None:
        """Dropout kernels launched (or captured) while on add the staged word to their seeds."""
        if self._seed_word is not None:
            torch.ops.llmtrain_hip.set_dropout_seed_offset(self._seed_word if on else None)

    # -- input handling --------------------------------------------------------------------

    @staticmethod
    def _signature(batches: list[dict[str, Any]]) -> tuple:
        return tuple(
            tuple(sorted((k, tuple(v.shape), v.dtype) for k, v in b.items() if torch.is_tensor(v))) for b in batches
        )

    def _graphable(self, batches: list[dict[str, Any]]) -> bool:
        if any("attention_mask" in b for b in batches):  # padding survived the all-ones drop
            return False
        return self._static is None or self._signature(batches) == self._signature(self._static)

    def _to_static(self, batches: list[dict[str, Any]]) -> None:
        if self._static is None:
            self._static = [
                {k: (v.to(self._device).clone() if torch.is_tensor(v) else v) for k, v in b.items()} for b in batches
            ]
            return
        for dst, src in zip(self._static, batches):
            for k, v in src.items():
                if torch.is_tensor(v):
                    dst[k].copy_(v, non_blocking=True)

    # -- one optimizer step ----------------------------------------------------------------

    def step(self, host_batches: list[dict[str, Any]]) -> tuple[torch.Tensor, torch.Tensor]:
        """One optimizer step over ``host_batches`` (the micro-batches, CPU tensors, padding masks
        already dropped where all-ones); returns ``(mean loss, pre-clip grad norm)`` as device
        scalars that later steps do not overwrite."""
        self._stage_dropout(self._opt.steps_taken + 1)
        if self._calls < self._warmup or not self._graphable(host_batches):
            self._calls += 1
            self.eager_steps += 1
            self._kernels_read_word(True)
            try:
                return self._eager_on_stream(host_batches)
            finally:
                self._kernels_read_word(False)
        self._calls += 1
        if self._graph is None:
            self._kernels_read_word(True)
            try:
                self._capture(host_batches)
            finally:
                self._kernels_read_word(False)
        else:
            self._to_static(host_batches)
            self._opt.stage_graph_step()
        assert self._graph is not None and self._out is not None
        self._graph.replay()
        self.replays += 1
        self._after()
        loss, norm = self._out
        return loss.clone(), norm.clone()

    def _eager_on_stream(self, host_batches: list[dict[str, Any]]) -> tuple[torch.Tensor, torch.Tensor]:
        # on the capture stream, so per-stream library state (hipBLASLt handles/workspaces) exists
        # before the capture
        cur = torch.cuda.current_stream(self._device)
        self._stream.wait_stream(cur)
        with torch.cuda.stream(self._stream):
            dev = [{k: (v.to(self._device, non_blocking=True) if torch.is_tensor(v) else v) for k, v in b.items()}
                   for b in host_batches]
            out = self._eager(dev)
        cur.wait_stream(self._stream)
        return out

    def _capture(self, host_batches: list[dict[str, Any]]) -> None:
        self._to_static(host_batches)
        self._opt.stage_graph_step()  # this step's counter and scalars (read by the first replay)
        torch.cuda.synchronize(self._device)
        torch.cuda.empty_cache()  # the eager warm-up's cached blocks: the graph gets its own pool
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=self._stream):
            out = self._body(self._static)  # type: ignore[arg-type]
        self._graph, self._out = graph, out
        logger.info("trainer: captured the optimizer step as a hipGraph (%d micro-batches)", len(host_batches))
