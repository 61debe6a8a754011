"""Flat, contiguous parameter/gradient storage for the fused training path.

Every trainable parameter of a model is re-pointed at a view into ONE fp32 master buffer, its
``.grad`` at a view into ONE fp32 gradient buffer, and a compute-dtype (bf16) *shadow* buffer
mirrors the master weights for the GEMMs.  The segments are laid out in the order the fused
backward produces gradients (last layer first), so a data-parallel gradient bucket is simply a
contiguous slice of the gradient buffer: RCCL all-reduces it in place — no pack/unpack copies
(reference DDP Reducer buckets, ``training/trainer.py:86-91``, copy every gradient twice).

The last segment may carry *row padding* in the shadow buffer only (the tied token embedding /
LM head is padded from V=50257 to a multiple of 64 rows so the vocab GEMM and the fused
cross-entropy see MFMA-friendly shapes); the padding rows stay zero forever.

Parameters stay ordinary ``nn.Parameter`` objects, so ``model.parameters()``, ``state_dict()``
(fp32 master values, reference checkpoint layout) and ``clip_grad_norm_`` keep working.
"""

from __future__ import annotations

from collections.abc import Sequence
from dataclasses import dataclass

import torch
from torch import nn

__all__ = ["FlatParamStore", "Segment"]


@dataclass(frozen=True)
class Segment:
    """A named group of parameters that becomes gradient-ready at the same point in backward."""

    name: str
    start: int  # element offset in the flat buffers
    numel: int


class FlatParamStore:
    """Owns the flat master/grad/shadow buffers for an ordered list of parameter groups.

    Args:
        groups: ``[(segment_name, [param, ...]), ...]`` in gradient-production order.
        shadow_dtype: dtype of the compute copy (bf16 on GPU).
        pad_last_rows: pad the LAST parameter's leading dim to a multiple of this in the shadow.
    """

    def __init__(
        self,
        groups: Sequence[tuple[str, Sequence[nn.Parameter]]],
        *,
        shadow_dtype: torch.dtype,
        pad_last_rows: int = 1,
    ) -> None:
        params: list[nn.Parameter] = []
        seen: set[int] = set()
        segments: list[Segment] = []
        offset = 0
        for name, plist in groups:
            start = offset
            for p in plist:
                if id(p) in seen:
                    raise ValueError(f"parameter listed twice in flat layout (segment {name})")
                seen.add(id(p))
                params.append(p)
                offset += p.numel()
            segments.append(Segment(name, start, offset - start))
        if not params:
            raise ValueError("FlatParamStore needs at least one parameter")
        device = params[0].device
        self.params = params
        self.segments = segments
        self.numel = offset
        self.device = device
        self.shadow_dtype = shadow_dtype

        last = params[-1]
        rows = last.shape[0]
        padded_rows = -(-rows // pad_last_rows) * pad_last_rows
        self.last_padded_rows = padded_rows
        self.shadow_numel = offset + (padded_rows - rows) * (last.numel() // rows)

        self.master = torch.empty(offset, dtype=torch.float32, device=device)
        self.grad = torch.zeros(offset, dtype=torch.float32, device=device)
        self.shadow = torch.zeros(self.shadow_numel, dtype=shadow_dtype, device=device)
        self._offsets: dict[int, int] = {}

        cursor = 0
        with torch.no_grad():
            for p in params:
                n = p.numel()
                self.master[cursor : cursor + n].copy_(p.detach().reshape(-1).float())
                p.data = self.master[cursor : cursor + n].view_as(p)
                p.grad = self.grad[cursor : cursor + n].view_as(p)
                self._offsets[id(p)] = cursor
                cursor += n
        self._synced_version = -1
        self.sync_shadow()

    # -- views -----------------------------------------------------------------------------

    def offset_of(self, p: torch.Tensor) -> int:
        return self._offsets[id(p)]

    def owns(self, p: torch.Tensor) -> bool:
        return id(p) in self._offsets

    def shadow_of(self, p: torch.Tensor, *, padded: bool = False) -> torch.Tensor:
        """Compute-dtype view of parameter ``p`` (``padded`` only for the last parameter)."""
        off = self._offsets[id(p)]
        if padded:
            if p is not self.params[-1]:
                raise ValueError("only the last parameter of the layout is row-padded")
            rows = self.last_padded_rows
            cols = p.numel() // p.shape[0]
            return self.shadow[off : off + rows * cols].view(rows, cols)
        return self.shadow[off : off + p.numel()].view_as(p)

    def grad_of(self, p: torch.Tensor) -> torch.Tensor:
        off = self._offsets[id(p)]
        return self.grad[off : off + p.numel()].view_as(p)

    def segment(self, name: str) -> Segment:
        for seg in self.segments:
            if seg.name == name:
                return seg
        raise KeyError(name)

    # -- state maintenance -----------------------------------------------------------------

    def reattach_grads(self) -> None:
        """Re-point ``p.grad`` at the flat buffer (after a caller set grads to None)."""
        for p in self.params:
            off = self._offsets[id(p)]
            if p.grad is None or p.grad.data_ptr() != self.grad[off:].data_ptr():
                p.grad = self.grad[off : off + p.numel()].view_as(p)

    def zero_grad(self) -> None:
        self.grad.zero_()
        self.reattach_grads()

    def version(self) -> int:
        """Monotone counter over every in-place write to the master weights.

        ``p.data = view`` gives each parameter its own autograd version counter, so the sum
        over the parameters (plus the master buffer itself) is what moves on ``p.copy_``.
        """
        return self.master._version + sum(p._version for p in self.params)

    def shadow_is_stale(self) -> bool:
        return self._synced_version != self.version()

    def sync_shadow(self, *, force: bool = False) -> None:
        """Refresh the compute copy if the master weights changed since the last sync.

        Any in-place write to a parameter (``load_state_dict``, user code) bumps a version
        counter (:meth:`version`), so staleness is detected without hashing.
        """
        if force or self.shadow_is_stale():
            with torch.no_grad():
                self.shadow[: self.numel].copy_(self.master)
            self.mark_shadow_synced()

    def mark_shadow_synced(self) -> None:
        self._synced_version = self.version()
