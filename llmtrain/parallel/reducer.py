"""Bucketed gradient all-reduce over the flat gradient buffer of the fused engine.

This is the MI355X replacement for torch's DDP Reducer on the fused path (reference wraps the
model in ``DistributedDataParallel`` at ``training/trainer.py:86-91``):

* **zero-copy buckets** — gradients already live in one flat fp32 buffer laid out in backward
  order (:class:`llmtrain.runtime.flat.FlatParamStore`), so a bucket is a contiguous slice that
  RCCL reduces in place; no bucket pack/unpack kernels, no ``gradient_as_bucket_view`` dance;
* **overlap** — the engine calls :meth:`FlatDataParallel._on_segment_ready` as soon as a
  layer's gradients are final; when a bucket's last segment arrives its ``all_reduce`` is
  issued from the reducer's comm stream, ordered after the producing kernels by a stream wait,
  while the backward of the earlier layers continues on the compute streams;
* **observable** — per-bucket ready / start / end events (:meth:`bucket_timeline`) show how long a
  bucket queued and how long RCCL took beside the saturating compute streams, not just the
  exposed tail after the backward (:meth:`exposed_comm_ms`);
* **xGMI sizing** — on a ring each GPU moves ``2(n-1)/n · S`` bytes per bucket over one link,
  so buckets are sized for link latency amortisation (default 64 MiB, two GPT-2-small blocks)
  rather than for NVSwitch;
* **no buffer broadcasts** — the constant ``causal_mask`` buffers are never re-broadcast
  (SURVEY Q18); parameters are broadcast once from rank 0 at wrap time as a single flat tensor;
* **no_sync()** — gradient accumulation micro-steps skip communication exactly like DDP;
* **comm stream at high priority** — RCCL's workgroups are dispatched ahead of the compute
  stream's queued GEMM tiles instead of waiting for a whole kernel's worth of them to drain;
* **bucket-wise gradient norm** — as soon as a bucket's all-reduce is done, its squared L2 norm is
  summed on the comm stream (:meth:`grad_sumsq`), so after the backward the clip coefficient needs
  only the last (tied-embedding) bucket's partial instead of a pass over every gradient.
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
        self._trace: list[list[Any]] = []  # this step's [bucket, ready, start, end] rows
        self._trace_hist: deque[list[list[Any]]] = deque(maxlen=64)
        # GPU: collectives are issued from a dedicated comm stream (see _launch), created at the highest
        # priority the device offers: with one compute stream holding every CU, a default-priority
        # stream's RCCL workgroups would queue behind the GEMM tiles already waiting for a CU
        self._comm = (
            torch.cuda.Stream(device=self._store.grad.device, priority=torch.cuda.Stream.priority_range()[1])
            if self._store.grad.is_cuda else None
        )
        # squared L2 norm of each bucket's reduced gradient (written on the comm stream / at finish)
        self._sq = torch.zeros(len(self.buckets), dtype=torch.float32, device=self._store.grad.device)
        self._sq_ready = False
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
            self._sq_ready = False

    def _on_segment_ready(self, segment: str) -> None:
        if not (self._sync and self._armed):
            return
        idx = self._bucket_of[segment]
        self._remaining[idx] -= 1
        if self._remaining[idx] == 0:
            self._launch(self.buckets[idx])

    def _launch(self, bucket: Bucket) -> None:
        """All-reduce one bucket.  On a GPU the collective is issued from the reducer's own comm
        stream, which first waits for the producing stream (the engine's weight-gradient side
        stream, already joined with the main stream): a bf16 payload is cast and cast back there,
        so neither compute stream ever queues communication work.  Three timing events per
        bucket — ``ready`` on the producing stream, ``start`` / ``end`` on the comm stream around
        the collective — feed :meth:`bucket_timeline` (how long a bucket waited behind earlier
        buckets, and how long RCCL took while the compute streams held the CUs)."""
        view = self._store.grad[bucket.start : bucket.start + bucket.numel]
        op = dist.ReduceOp.AVG if self._avg_native else dist.ReduceOp.SUM
        if self._comm is None:  # CPU / gloo: host timestamps; the collective runs asynchronously
            staged = view.to(self.reduce_dtype) if self._staged_dtype(view) else None
            payload = view if staged is None else staged
            t_ready = time.perf_counter()
            work = dist.all_reduce(payload, op=op, group=self._pg, async_op=True)
            self._works.append((bucket, work, staged))
            self._trace.append([bucket, t_ready, None, None])
            return
        producer = torch.cuda.current_stream()
        ready, start, end = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        ready.record(producer)
        self._comm.wait_stream(producer)
        with torch.cuda.stream(self._comm):
            start.record()
            staged = view.to(self.reduce_dtype) if self._staged_dtype(view) else None
            payload = view if staged is None else staged
            work = dist.all_reduce(payload, op=op, group=self._pg, async_op=True)
            if self._avg_native:
                work.wait()  # RCCL: the comm stream waits for the collective (the host does not)
                if staged is not None:
                    view.copy_(staged)
                self._bucket_sumsq(bucket, view)
                end.record()
                work = None
        self._works.append((bucket, work, staged))
        self._trace.append([bucket, ready, start, end])

    def _bucket_sumsq(self, bucket: Bucket, view: torch.Tensor) -> None:
        """This bucket's squared norm into its slot, on the stream that finished its reduction."""
        from llmtrain import ops

        self._sq[bucket.index : bucket.index + 1].copy_(ops.sumsq(view).reshape(1))

    def grad_sumsq(self) -> torch.Tensor | None:
        """Squared global L2 norm of the reduced gradients of the last synchronised step (device
        scalar, after :meth:`finish_gradient_sync`), summed from the per-bucket partials in bucket
        order; ``None`` when the last step did not synchronise (accumulation micro-steps)."""
        return self._sq.sum() if self._sq_ready else None

    def _staged_dtype(self, view: torch.Tensor) -> bool:
        return self.reduce_dtype is not None and self.reduce_dtype != view.dtype

    def finish_gradient_sync(self) -> None:
        """Wait for every launched bucket and finalise averaging (stream-side on RCCL: the
        compute stream waits on the comm stream, the host does not block).

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
        if self._comm is not None:
            torch.cuda.current_stream().wait_stream(self._comm)
        for i, (bucket, work, staged) in enumerate(self._works):
            if work is None:
                continue
            work.wait()
            view = self._store.grad[bucket.start : bucket.start + bucket.numel]
            if staged is not None:
                view.copy_(staged)
            if not self._avg_native:
                view.div_(self.world_size)
            self._bucket_sumsq(bucket, view)
            if on_gpu:  # gloo on GPU tensors (a rehearsal): completion seen at this wait, an upper bound
                self._trace[i][3].record()
            else:
                self._trace[i][3] = time.perf_counter()
        if on_gpu:
            t_end = torch.cuda.Event(enable_timing=True)
            t_end.record()
            self._exposed = (t_start, t_end)
        else:
            self._exposed = 1000.0 * (time.perf_counter() - t_host)
        self._exposed_hist.append(self._exposed)
        self._trace_hist.append(self._trace)
        self._trace = []
        self._works.clear()
        self._armed = False
        self._sq_ready = True

    def bucket_timeline(self) -> list[list[dict[str, float]]]:
        """Per synchronised step since the last call (oldest first, at most 64), per bucket:
        ``mib`` (payload on the wire); on a GPU ``queue_ms`` (ready on the producing stream -> the comm stream started
        it: waiting behind earlier buckets), ``comm_ms`` (start -> end: the collective itself,
        including any wait for CUs the compute streams hold), ``ready_ms`` (ready, relative to
        the step's first ready bucket); on the host path ``ready_to_done_ms``.  Synchronises on
        the newest events — call at log intervals only.  Clears the history."""
        out = []
        wire = self.reduce_dtype or self._store.grad.dtype
        elem = torch.empty((), dtype=wire).element_size()
        for trace in self._trace_hist:
            rows = []
            first = trace[0][1] if trace else None
            for bucket, ready, start, end in trace:
                row: dict[str, float] = {"mib": round(bucket.numel * elem / 2**20, 2)}
                if isinstance(ready, float):
                    if end is not None:
                        row["ready_to_done_ms"] = 1000.0 * (end - ready)
                else:
                    end.synchronize()
                    row["ready_ms"] = float(first.elapsed_time(ready))
                    row["queue_ms"] = float(ready.elapsed_time(start))
                    row["comm_ms"] = float(start.elapsed_time(end))
                rows.append(row)
            out.append(rows)
        self._trace_hist.clear()
        return out

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
