"""Bucketed gradient all-reduce over the flat gradient buffer of the fused engine.

This is the MI355X replacement for torch's DDP Reducer on the fused path (reference wraps the
model in ``DistributedDataParallel`` at ``training/trainer.py:86-91``):

* **zero-copy buckets** — gradients already live in one flat fp32 buffer laid out in backward
  order (:class:`llmtrain.runtime.flat.FlatParamStore`), so a bucket is a contiguous slice that
  RCCL reduces in place; no bucket pack/unpack kernels, no ``gradient_as_bucket_view`` dance;
* **overlap** — the engine calls :meth:`FlatDataParallel._on_segment_ready` as soon as a
  layer's gradients are final; when a bucket's last segment arrives its ``all_reduce`` is
  issued asynchronously (RCCL runs it on its own stream, ordered after the producing kernels
  by an event) while the backward of the earlier layers continues on the compute stream;
* **xGMI sizing** — on a ring each GPU moves ``2(n-1)/n · S`` bytes per bucket over one link,
  so buckets are sized for link latency amortisation (default 64 MiB, two GPT-2-small blocks)
  rather than for NVSwitch;
* **no buffer broadcasts** — the constant ``causal_mask`` buffers are never re-broadcast
  (SURVEY Q18); parameters are broadcast once from rank 0 at wrap time as a single flat tensor;
* **no_sync()** — gradient accumulation micro-steps skip communication exactly like DDP.
"""

from __future__ import annotations

import contextlib
import logging
import time
from collections import deque
from collections.abc import Iterator
from dataclasses import dataclass
from typing import Any

import torch
import torch.distributed as dist
from torch import nn

__all__ = ["Bucket", "FlatDataParallel", "plan_buckets"]

logger = logging.getLogger(__name__)


@dataclass(frozen=True)
class Bucket:
    index: int
    start: int
    numel: int
    segments: tuple[str, ...]


def plan_buckets(segments, *, cap_bytes: int, elem_bytes: int = 4) -> list[Bucket]:
    """Greedily merge consecutive segments (backward order) until a bucket reaches ``cap_bytes``."""
    buckets: list[Bucket] = []
    cur: list[Any] = []
    size = 0
    for seg in segments:
        cur.append(seg)
        size += seg.numel * elem_bytes
        if size >= cap_bytes:
            buckets.append(_make_bucket(len(buckets), cur))
            cur, size = [], 0
    if cur:
        buckets.append(_make_bucket(len(buckets), cur))
    return buckets


def _make_bucket(index: int, segs: list[Any]) -> Bucket:
    start = segs[0].start
    end = segs[-1].start + segs[-1].numel
    for a, b in zip(segs, segs[1:]):
        if a.start + a.numel != b.start:
            raise ValueError("bucket segments must be contiguous in the flat buffer")
    return Bucket(index, start, end - start, tuple(s.name for s in segs))


class FlatDataParallel(nn.Module):
    """Data-parallel wrapper for a model prepared with a fused engine (``model.engine``)."""

    def __init__(
        self,
        module: nn.Module,
        *,
        process_group: Any = None,
        bucket_cap_mb: float = 64.0,
        reduce_dtype: torch.dtype | None = None,
        broadcast_parameters: bool = True,
    ) -> None:
        super().__init__()
        engine = getattr(module, "engine", None)
        if engine is None:
            raise ValueError("FlatDataParallel needs a model with a prepared fused engine")
        self.module = module
        self._engine = engine
        self._store = engine.store
        self._pg = process_group
        self.world_size = dist.get_world_size(process_group)
        self._avg_native = dist.get_backend(process_group) == "nccl"
        self.reduce_dtype = reduce_dtype
        self.buckets = plan_buckets(self._store.segments, cap_bytes=int(bucket_cap_mb * 2**20))
        self._bucket_of = {name: b.index for b in self.buckets for name in b.segments}
        self._remaining: list[int] = []
        self._works: list[tuple[Bucket, Any, torch.Tensor | None]] = []
        self._sync = True
        self._armed = False
        self._exposed: tuple[Any, Any] | float | None = None
        self._exposed_hist: deque[tuple[Any, Any] | float] = deque(maxlen=256)
        engine.grad_ready = self._on_segment_ready
        if broadcast_parameters and self.world_size > 1:
            with torch.no_grad():
                dist.broadcast(self._store.master, src=0, group=process_group)
            self._store.sync_shadow(force=True)
        logger.info(
            "FlatDataParallel: world=%d buckets=%d sizes(MiB)=%s",
            self.world_size,
            len(self.buckets),
            [round(b.numel * 4 / 2**20, 2) for b in self.buckets],
        )

    # -- module protocol -------------------------------------------------------------------

    def forward(self, *args: Any, **kwargs: Any) -> Any:
        return self.module(*args, **kwargs)

    @property
    def engine(self) -> Any:
        return self._engine

    def fused_loss(self, input_ids, labels, attention_mask=None) -> torch.Tensor:
        self._arm()
        return self.module.fused_loss(input_ids, labels, attention_mask)

    @contextlib.contextmanager
    def no_sync(self) -> Iterator[None]:
        previous, self._sync = self._sync, False
        try:
            yield
        finally:
            self._sync = previous

    # -- reduction -------------------------------------------------------------------------

    def _arm(self) -> None:
        if self._sync:
            if self._works:
                raise RuntimeError("previous gradient all-reduce was not finished")
            self._remaining = [len(b.segments) for b in self.buckets]
            self._armed = True

    def _on_segment_ready(self, segment: str) -> None:
        if not (self._sync and self._armed):
            return
        idx = self._bucket_of[segment]
        self._remaining[idx] -= 1
        if self._remaining[idx] == 0:
            self._launch(self.buckets[idx])

    def _launch(self, bucket: Bucket) -> None:
        view = self._store.grad[bucket.start : bucket.start + bucket.numel]
        staged = None
        payload = view
        if self.reduce_dtype is not None and self.reduce_dtype != view.dtype:
            staged = view.to(self.reduce_dtype)
            payload = staged
        op = dist.ReduceOp.AVG if self._avg_native else dist.ReduceOp.SUM
        work = dist.all_reduce(payload, op=op, group=self._pg, async_op=True)
        self._works.append((bucket, work, staged))

    def finish_gradient_sync(self) -> None:
        """Wait (stream-side on RCCL) for every launched bucket and finalise averaging.

        The wait is bracketed by timing events on the compute stream: their distance is the
        *exposed* communication time — how long the optimizer waited for all-reduces still in
        flight after the backward's last kernel (:meth:`exposed_comm_ms`)."""
        if not self._armed:
            return
        if any(r != 0 for r in self._remaining):
            raise RuntimeError(f"gradient buckets never completed: {self._remaining}")
        on_gpu = self._store.grad.is_cuda
        if on_gpu:
            t_start = torch.cuda.Event(enable_timing=True)
            t_start.record()
        else:
            t_host = time.perf_counter()
        for bucket, work, staged in self._works:
            work.wait()
            view = self._store.grad[bucket.start : bucket.start + bucket.numel]
            if staged is not None:
                view.copy_(staged)
            if not self._avg_native:
                view.div_(self.world_size)
        if on_gpu:
            t_end = torch.cuda.Event(enable_timing=True)
            t_end.record()
            self._exposed = (t_start, t_end)
        else:
            self._exposed = 1000.0 * (time.perf_counter() - t_host)
        self._exposed_hist.append(self._exposed)
        self._works.clear()
        self._armed = False

    def exposed_comm_ms(self) -> float | None:
        """Exposed all-reduce time of the last synchronised step in ms (``None`` before the first).
        Reading it synchronises on that step's end event — call it at log intervals only."""
        return None if self._exposed is None else self._resolve(self._exposed)

    def drain_exposed_comm_ms(self) -> list[float]:
        """Exposed all-reduce ms of every step synchronised since the last drain (oldest first,
        at most 256); clears the history.  Synchronises on the newest step's end event."""
        out = [self._resolve(ex) for ex in self._exposed_hist]
        self._exposed_hist.clear()
        return out

    @staticmethod
    def _resolve(ex: tuple[Any, Any] | float) -> float:
        if isinstance(ex, float):
            return ex
        ex[1].synchronize()
        return float(ex[0].elapsed_time(ex[1]))
