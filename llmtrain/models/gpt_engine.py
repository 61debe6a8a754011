"""Fused MI355X execution engine for :class:`llmtrain.models.gpt.GPT`.

The engine runs a whole forward + loss, and later the whole backward, as one explicitly
scheduled sequence of kernels instead of an autograd graph of small ops:

forward (per block; ``M = B*T`` tokens, ``d`` model width, residual stream kept in fp32)::

    x_s, h1  = add_layernorm(x, delta)            # HIP: residual add fused into LN, bf16 out
    qkv      = h1 @ Wqkv^T + b                    # hipBLASLt (bias epilogue), bf16
    att, lse = flash_attn_fwd(qkv)                # HIP: gfx950 MFMA, packed qkv, causal
    y        = att @ Wo^T + b                     # hipBLASLt
    x_m, h2  = add_layernorm(x_s, y)              # HIP
    u        = h2 @ Wfc^T + b                     # hipBLASLt
    g        = gelu(u)                            # HIP (exact erf GELU)
    delta    = g @ Wproj^T + b                    # hipBLASLt  (added by the next LN)

Dropout (reference ``nn.Dropout`` after the embeddings, on the attention probabilities and on
both residual branches, active in train mode) is fused into those kernels: each site's keep-mask
is a counter-based hash of (step seed, site, element index) — see ``csrc/common.h`` — so the
backward regenerates it instead of storing it.  Sites per forward: 0 = embedding, then per block
``i``: ``1+3i`` attention-output branch, ``2+3i`` attention probabilities, ``3+3i`` MLP branch.

then ``ln_f`` (+ the last residual add), the tied LM head GEMM against a vocab-padded bf16
shadow (50257 → 50304 rows) and a fused softmax-cross-entropy kernel that produces the per-row
loss AND overwrites the logits with their gradient in the same pass (the logits are dead after
the loss, so the backward never re-reads them as logits).

backward mirrors it in reverse with fp32 weight-gradient GEMMs that accumulate straight into
the flat gradient buffer (``addmm(out_dtype=fp32, beta=1)``), LayerNorm backward kernels that
also emit the bf16 copy of ``dx`` and the projection-bias column sums, and a flash-attention
backward.  The loss-gradient scale (``1/grad_accum``) is folded into the first backward kernel
through a device scalar — no host sync anywhere in the step.

After each block's gradients are final the engine calls ``grad_ready(segment_name)`` so a
data-parallel reducer (:mod:`llmtrain.parallel.reducer`) can all-reduce that bucket while the
remaining backward runs (reference: torch DDP Reducer hooks, ``training/trainer.py:86-91``).

Reference call sites replaced: ``models/gpt.py:49-74`` (attention), ``:86-105`` (LN/MLP),
``:176-184`` (embeddings, ln_f, lm_head), ``:256-269`` (cross-entropy + masked mean).
"""

from __future__ import annotations

import os
import warnings
from collections.abc import Callable
from dataclasses import dataclass, field
from typing import Any

import torch

from llmtrain import ops
from llmtrain.ops.reference import dropout_site_seed
from llmtrain.runtime.flat import FlatParamStore

__all__ = ["FusedGPTEngine"]

VOCAB_PAD = 64  # pad the LM-head rows to a multiple of the MFMA-friendly tile


def _mm(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return torch.mm(a, b)


_WGRAD_MODE: dict[str, str] = {}


def accumulate_wgrad(dst: torch.Tensor, dy: torch.Tensor, x: torch.Tensor) -> None:
    """``dst (fp32) += dy^T @ x`` with low-precision operands and fp32 accumulation.

    Uses ``addmm(..., out_dtype=float32)`` in place (hipBLASLt with an fp32 C/D matrix) when the
    backend supports it, else a fp32-output GEMM plus an add.
    """
    if dy.dtype == torch.float32:
        dst.addmm_(dy.t(), x)
        return
    key = str(dst.device.type)
    mode = _WGRAD_MODE.get(key)
    if mode in (None, "inplace"):
        try:
            torch.addmm(dst, dy.t(), x, out_dtype=torch.float32, out=dst)
            _WGRAD_MODE[key] = "inplace"
            return
        except (RuntimeError, TypeError):
            if mode == "inplace":
                raise
            _WGRAD_MODE[key] = "mm"
    if dst.device.type != "cuda":  # CPU (tests): no fp32-output mm for bf16 operands
        dst.add_(torch.mm(dy.t().float(), x.float()))
        return
    dst.add_(torch.mm(dy.t(), x, out_dtype=torch.float32))


@dataclass
class _BlockActs:
    xs: torch.Tensor  # fp32 residual stream entering the attention sub-block
    h1: torch.Tensor
    mu1: torch.Tensor
    rs1: torch.Tensor
    qkv: torch.Tensor
    att: torch.Tensor
    lse: torch.Tensor
    xm: torch.Tensor  # fp32 residual stream entering the MLP sub-block
    h2: torch.Tensor
    mu2: torch.Tensor
    rs2: torch.Tensor
    u: torch.Tensor
    g: torch.Tensor


@dataclass
class _StepState:
    ids: torch.Tensor
    bsz: int
    seqlen: int
    blocks: list[_BlockActs] = field(default_factory=list)
    xf: torch.Tensor | None = None
    hf: torch.Tensor | None = None
    muf: torch.Tensor | None = None
    rsf: torch.Tensor | None = None
    dlogits: torch.Tensor | None = None
    drop_p: float = 0.0
    drop_seed: int = 0
    # key-padding mask (reference gpt.py:60-64, 73-74): the attention kernels' key masks and the
    # [M, 1] row keep-factor that zeroes the attention branch of padded query positions
    key_masks: tuple[torch.Tensor, torch.Tensor] | None = None
    keep_col: torch.Tensor | None = None

    def site(self, k: int) -> tuple[float, int]:
        """``(p, site_seed)`` of dropout site ``k`` for this forward (``(0, 0)`` = off)."""
        if self.drop_p <= 0.0:
            return (0.0, 0)
        return (self.drop_p, dropout_site_seed(self.drop_seed, k))


class _FusedLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, engine, ids, labels, mask):  # type: ignore[override]
        loss, state = engine._forward(ids, labels, mask, keep=True)
        ctx.engine = engine
        ctx.state = state
        return loss

    @staticmethod
    def backward(ctx, grad_out):  # type: ignore[override]
        state, ctx.state = ctx.state, None
        ctx.engine._backward(state, grad_out)
        return None, None, None, None, None


RESIDUAL_MODES = ("fp32", "bf16_grad", "bf16")
MLP_STORE_GD_MAX_D = 1024  # default mlp_store "gd" up to this d_model, "u" above


class FusedGPTEngine:
    """Owns the flat parameter store of a GPT and runs its fused forward/backward."""

    SIDE_LAG = 2  # blocks of side-stream GEMM operands kept alive before the main stream fences them

    def __init__(
        self, model: Any, *, compute_dtype: torch.dtype = torch.bfloat16, residual: str | None = None,
        mlp_store: str | None = None,
    ) -> None:
        self.model = model
        self.compute_dtype = compute_dtype
        # storage of the residual stream (x, xs, xm: the LayerNorm inputs) and of its gradient
        # (model.extra.residual_dtype): "fp32" (the reference's precision; the default with an fp32
        # compute dtype), "bf16_grad" (the backward's residual-gradient stream in bf16: LayerNorm
        # backward moves 10 instead of 16 bytes per element) or "bf16" (both streams in bf16:
        # 8 + 8 instead of 12 + 16; the default with the bf16 compute dtype, as in Megatron-style
        # bf16 training without fp32 residual connections).  The adds, LayerNorm statistics and row
        # math stay fp32 in registers either way; the bf16 forms round the stored values.  Measured
        # (docs/round6.md §4): GPT-2 124M +3.6 % tok/s, -4.7 GiB peak, 1,500-step validation loss
        # within the fp32-residual path's seed spread
        if residual is None:
            residual = "bf16" if compute_dtype == torch.bfloat16 else "fp32"
        if residual not in RESIDUAL_MODES:
            raise ValueError(f"residual_dtype must be one of {RESIDUAL_MODES}, not {residual!r}")
        if residual != "fp32" and compute_dtype != torch.bfloat16:
            raise ValueError("a bf16 residual stream needs the bf16 compute dtype")
        self.residual = residual
        self.res_dtype = torch.bfloat16 if residual == "bf16" else torch.float32
        self.grad_dtype = torch.float32 if residual == "fp32" else torch.bfloat16
        self.blocks = list(model.blocks)
        self.n_heads = model.n_heads
        self.head_dim = model.d_model // model.n_heads
        self.vocab = model.vocab_size
        self.eps = model.ln_f.eps
        for blk in self.blocks:
            if blk.ln_1.eps != self.eps or blk.ln_2.eps != self.eps:
                raise ValueError("fused engine assumes one LayerNorm eps for the whole model")

        groups: list[tuple[str, list[torch.nn.Parameter]]] = [
            ("ln_f", [model.ln_f.weight, model.ln_f.bias])
        ]
        for i in reversed(range(len(self.blocks))):
            b = self.blocks[i]
            groups.append(
                (
                    f"block{i}",
                    [
                        b.mlp_proj.weight, b.mlp_proj.bias, b.mlp_fc.weight, b.mlp_fc.bias,
                        b.ln_2.weight, b.ln_2.bias, b.attn.out_proj.weight, b.attn.out_proj.bias,
                        b.attn.qkv_proj.weight, b.attn.qkv_proj.bias, b.ln_1.weight, b.ln_1.bias,
                    ],
                )
            )
        emb = [model.position_embedding.weight]
        if model.tie_embeddings:
            emb.append(model.token_embedding.weight)
        else:
            emb += [model.token_embedding.weight, model.lm_head.weight]
        groups.append(("embed", emb))
        self.segment_order = [name for name, _ in groups]
        self.store = FlatParamStore(groups, shadow_dtype=compute_dtype, pad_last_rows=VOCAB_PAD)
        self.grad_ready: Callable[[str], None] | None = None
        # per-forward dropout base seed provider (None: one draw from torch's CPU generator)
        self.drop_seed_source: Callable[[], int] | None = None
        self._anchor = torch.zeros((), requires_grad=True, device=self.store.device)
        # weight-gradient GEMMs on a second HIP stream beside the main stream's dX GEMMs and
        # bandwidth-bound kernels (LLMTRAIN_WGRAD_STREAM=1).  Off by default since round 4: the
        # ping-pong weight-gradient kernel takes 2 x 236 registers of every SIMD it lands on, so
        # nothing of the main stream co-resides with it and the two streams only time-share the
        # chip; one stream measured +0.9 % at micro-batch 128 and +1.0 % at 32 (same box,
        # profiles/r4/ab_side_stream_vs_one_stream_mb*.txt), and is the deterministic schedule.
        self.wgrad_stream_enabled = os.environ.get("LLMTRAIN_WGRAD_STREAM", "0") != "0"
        # hand-written MFMA GEMM (csrc/gemm_fused.hip) where it beats hipBLASLt: qkv and attention
        # output projections (forward and dX), the fc forward with bias + GELU in its epilogue, the
        # MLP projection dX with the GELU backward + fc-bias gradient in its epilogue
        # (LLMTRAIN_FUSED_GEMM=0: hipBLASLt everywhere + separate GELU passes)
        self.fused_gemm = os.environ.get("LLMTRAIN_FUSED_GEMM", "1") != "0"
        # what the MLP keeps for its backward (model.extra.mlp_store): "u", the fc pre-activation
        # (the dX epilogue evaluates gelu'(u)), or "gd", gelu'(u) itself, formed by the fc GEMM's
        # epilogue from the same erf as gelu(u) (the dX epilogue then multiplies by a stored value)
        if mlp_store is None:
            # measured (docs/round6.md §8): "gd" +0.5 % at GPT-2 124M (d 768: the fc forward's fused
            # epilogue costs less than the erf it saves the dX), -0.7 % at GPT-2 XL (d 1600: the
            # library's fc forward + GELU pass stays ahead of the fused fc forward)
            mlp_store = "gd" if self.fused_gemm and model.d_model <= MLP_STORE_GD_MAX_D else "u"
        if mlp_store not in ("u", "gd"):
            raise ValueError(f"mlp_store must be 'u' or 'gd', not {mlp_store!r}")
        self.mlp_store = mlp_store
        self.markers = os.environ.get("LLMTRAIN_ROCTX", "0") == "1" and self.store.device.type == "cuda"
        # set by a Trainer with run.deterministic: warn once if a step runs outside its kernel policy
        self.expect_deterministic = False
        self._warned_policy = False
        self._side: torch.cuda.Stream | None = None
        self._pending: list[torch.Tensor] = []  # operands of side-stream GEMMs of the current block
        self._held: list[tuple[Any, list[torch.Tensor]]] = []  # (side event, operands) per block

    # ------------------------------------------------------------------------------------

    @property
    def head_weight(self) -> torch.nn.Parameter:
        return self.model.lm_head.weight

    def _w(self, p: torch.Tensor) -> torch.Tensor:
        return self.store.shadow_of(p)

    def _g(self, p: torch.Tensor) -> torch.Tensor:
        return self.store.grad_of(p)

    def _wgrad(self, dst: torch.Tensor, dy: torch.Tensor, x: torch.Tensor, bias: torch.Tensor | None = None) -> None:
        """Block weight (and bias: ``bias += colsum(dy)``) gradients: the split-K MFMA kernel
        (``ops.wgrad_accum``) on GPU — it fills the chip on these M-deep reductions where hipBLASLt
        picks too few tiles, and sums the bias columns from the ``dy`` tiles it streams anyway.  On
        GPU it runs on the side stream after an event on the main stream (``dy``/``x`` are ready);
        the engine holds ``dy``/``x`` until the main stream has fenced the GEMM
        (:meth:`_retire_block`), so their memory is not reused before the side stream is done."""
        if not (dst.is_cuda and dy.dtype == torch.bfloat16):
            accumulate_wgrad(dst, dy, x)
            if bias is not None:
                ops.colsum_accum(dy, bias)
            return
        side = self._side_stream()
        if side is not None:
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                ops.wgrad_accum(dst, dy, x, bias=bias)
            self._pending.extend((dy, x))
        else:  # one stream: nothing runs beside it
            ops.wgrad_accum(dst, dy, x, bias=bias)

    def _retire_block(self) -> None:
        """End of one block's backward: fence its side-stream GEMMs with an event and release the
        operands of the GEMMs ``SIDE_LAG`` blocks back once the main stream has waited on their
        event (free then, since the side stream keeps far ahead of that lag).

        This replaces ``record_stream``: a record_stream'd block returns to the caching allocator
        only when a later allocation happens to poll its event, so every step mallocs fresh blocks
        — reserved memory grew to the device limit and each allocator retry (emptyCache + re-malloc)
        cost 5x throughput at micro-batch 128."""
        if self._side is None:
            return
        ev = torch.cuda.Event()
        ev.record(self._side)
        self._held.append((ev, self._pending))
        self._pending = []
        while len(self._held) > self.SIDE_LAG:
            old, _ = self._held.pop(0)
            torch.cuda.current_stream().wait_event(old)

    def _side_stream(self) -> torch.cuda.Stream | None:
        if not self.wgrad_stream_enabled or not self.store.device.type == "cuda" or ops.single_stream():
            return None
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.store.device)
        return self._side

    def _join_side(self) -> None:
        """Main stream waits for every weight-gradient GEMM issued so far (then their operands
        may be reused by the main stream's allocator)."""
        if self._side is not None:
            torch.cuda.current_stream().wait_stream(self._side)
        self._held.clear()
        self._pending = []

    def _linear(self, x: torch.Tensor, layer: torch.nn.Linear, *, fused: bool = False) -> torch.Tensor:
        w = self._w(layer.weight)
        b = None if layer.bias is None else self._w(layer.bias)
        if fused and self.fused_gemm:
            return ops.linear_fwd(x, w, b)
        return torch.mm(x, w.t()) if b is None else torch.addmm(b, x, w.t())

    def loss(self, ids: torch.Tensor, labels: torch.Tensor, mask: torch.Tensor | None) -> torch.Tensor:
        if not self.fused_gemm and self.store.device.type == "cuda":
            ops._det_fallback("every GEMM (LLMTRAIN_FUSED_GEMM=0)")
        if self.expect_deterministic and not self._warned_policy and self.store.device.type == "cuda" \
                and not ops.policy_state()[0]["deterministic"]:
            # a Trainer configured run.deterministic scopes its own steps (Trainer.kernel_policy);
            # driving its model directly runs the fast path's atomics unless the caller scopes it
            self._warned_policy = True
            warnings.warn(
                "run.deterministic is set for this model's Trainer but the process-wide kernel policy is "
                "the fast (atomic) one here: wrap direct engine use in trainer.kernel_policy() or "
                "llmtrain.ops.kernel_policy(True)", RuntimeWarning, stacklevel=3,
            )
        self.store.sync_shadow()
        if torch.is_grad_enabled():
            return _FusedLoss.apply(self._anchor, self, ids, labels, mask)
        loss, _ = self._forward(ids, labels, mask, keep=False)
        return loss

    def _push(self, name: str) -> None:
        """Open a roctx range (``torch.cuda.nvtx`` is roctx on ROCm) around an engine phase when
        ``LLMTRAIN_ROCTX=1``: ``rocprofv3 --marker-trace`` / torch.profiler then show the fused
        step per block instead of a flat kernel list."""
        if self.markers:
            torch.cuda.nvtx.range_push(name)

    def _pop(self) -> None:
        if self.markers:
            torch.cuda.nvtx.range_pop()

    # -- forward ---------------------------------------------------------------------------

    def _forward(self, ids, labels, mask, *, keep: bool):
        m = self.model
        bsz, seqlen = ids.shape
        n_tok = bsz * seqlen
        cdt = self.compute_dtype
        state = _StepState(ids=ids, bsz=bsz, seqlen=seqlen)
        if m.training and m.dropout > 0.0:
            # one host draw per forward from torch's (seeded, checkpointed) CPU generator
            state.drop_p = float(m.dropout)
            if self.drop_seed_source is not None:  # a hipGraph-captured step (training/graph_step.py)
                state.drop_seed = int(self.drop_seed_source())
            else:
                state.drop_seed = int(torch.randint(0, 2**31 - 1, (1,)).item())

        if mask is not None:
            # key padding (no host sync: a mask is taken as given; the trainer drops all-ones masks
            # on the host before they reach the device)
            valid = mask.reshape(-1).bool()  # nonzero = valid, like the reference's mask.bool()
            row_w = valid.float()
            row_w = row_w / row_w.sum().clamp_min(1.0)
            state.key_masks = ops.attn_key_masks(mask)
            state.keep_col = valid.reshape(-1, 1).to(cdt)
        else:
            row_w = torch.full((n_tok,), 1.0 / n_tok, dtype=torch.float32, device=ids.device)

        self._push("fwd.embed")
        x = ops.embedding_fwd(
            ids, m.token_embedding.weight, m.position_embedding.weight, dropout=state.site(0), out_dtype=self.res_dtype
        )
        self._pop()
        delta: torch.Tensor | None = None
        for i, blk in enumerate(self.blocks):
            self._push(f"fwd.block{i}")
            xs, h1, mu1, rs1 = ops.add_layernorm_fwd(
                x, delta, blk.ln_1.weight, blk.ln_1.bias, self.eps, cdt, dropout=state.site(3 * i)
            )  # site 3i = the previous block's MLP branch (unused for block 0: delta is None)
            qkv = self._linear(h1, blk.attn.qkv_proj, fused=True)
            att, lse = ops.attn_fwd(
                qkv, bsz, seqlen, self.n_heads, dropout=state.site(2 + 3 * i), key_masks=state.key_masks
            )
            y = self._linear(att, blk.attn.out_proj, fused=True)
            if state.keep_col is not None:  # padded query rows add nothing to the residual stream
                y = y * state.keep_col
            xm, h2, mu2, rs2 = ops.add_layernorm_fwd(
                xs, y, blk.ln_2.weight, blk.ln_2.bias, self.eps, cdt, dropout=state.site(1 + 3 * i)
            )
            if self.fused_gemm and self.mlp_store == "gd":  # keeps gelu'(u) for the backward (in "u")
                u, g = ops.linear_fwd_gelu_gd(h2, self._w(blk.mlp_fc.weight), self._w(blk.mlp_fc.bias))
            elif self.fused_gemm:  # bias + exact-erf GELU in the fc GEMM's epilogue
                u, g = ops.linear_fwd_gelu(h2, self._w(blk.mlp_fc.weight), self._w(blk.mlp_fc.bias))
            else:
                u = self._linear(h2, blk.mlp_fc)
                g = ops.gelu_fwd(u)
            delta = self._linear(g, blk.mlp_proj, fused=True)
            x = xm
            if keep:
                state.blocks.append(_BlockActs(xs, h1, mu1, rs1, qkv, att, lse, xm, h2, mu2, rs2, u, g))
            self._pop()
        n_layers = len(self.blocks)
        self._push("fwd.head_ce")
        xf, hf, muf, rsf = ops.add_layernorm_fwd(
            x, delta, m.ln_f.weight, m.ln_f.bias, self.eps, cdt, dropout=state.site(3 * n_layers)
        )
        head = self.store.shadow_of(self.head_weight, padded=True)
        logits = ops.head_logits(hf, head)  # [M, Vp]
        per_row = ops.cross_entropy_fwd_bwd(logits, labels.reshape(-1), self.vocab, row_w)
        loss = torch.dot(per_row, row_w)
        if keep:
            state.dlogits = logits
        self._pop()
        if keep:
            state.xf, state.hf, state.muf, state.rsf = xf, hf, muf, rsf
        return loss, state

    # -- backward --------------------------------------------------------------------------

    def _notify(self, segment: str) -> None:
        """A segment's gradients are final: hand it to the data-parallel reducer.  Its bucket holds
        side-stream (weight) and main-stream (bias, LayerNorm) gradients, so the collective is
        launched from the side stream after it has caught up with the main stream — RCCL then
        orders the all-reduce after both without stalling the main stream's next layer."""
        if self.grad_ready is None:
            return
        if self._side is not None:
            self._side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self._side):
                self.grad_ready(segment)
        else:
            self.grad_ready(segment)

    def _backward(self, st: _StepState, grad_out: torch.Tensor) -> None:
        go = grad_out.detach().reshape(()).float()
        dlogits = st.dlogits
        assert dlogits is not None and st.hf is not None
        head = self.store.shadow_of(self.head_weight, padded=True)
        self._push("bwd.head")
        # LM head: dhf = dlogits @ W ; dW += dlogits^T @ (go * hf), both on the main stream (the
        # tied [V, d] gradient is also written by the embedding backward at the end: one stream)
        dhf = ops.head_dx(dlogits, head)
        hf_scaled = ops.scale(st.hf, go)  # one fused pass on GPU (fp32 math, one rounding)
        if dlogits.is_cuda and dlogits.dtype == torch.bfloat16:
            # split-K MFMA kernel: 9.78 vs 10.34 ms for hipBLASLt's fp32-output GEMM at 128K tokens
            # (bench/head_wgrad.py; N = 50257 rows inside the 50304-wide padded logits)
            ops.wgrad_accum(self._g(self.head_weight), dlogits[:, : self.vocab], hf_scaled)
        else:
            accumulate_wgrad(self._g(self.head_weight), dlogits[:, : self.vocab], hf_scaled)
        del hf_scaled
        st.dlogits = None
        del dlogits
        self._pop()
        self._backward_blocks(st, go, dhf)

    def _backward_blocks(self, st: _StepState, go: torch.Tensor, dhf: torch.Tensor) -> None:
        """Final LayerNorm and the transformer blocks, last to first, then the embeddings."""
        m = self.model
        bsz, seqlen = st.bsz, st.seqlen
        self._push("bwd.ln_f")
        last = self.blocks[-1]
        n_layers = len(self.blocks)
        dx, dx_lp = ops.layernorm_bwd(
            dhf, st.xf, st.muf, st.rsf, m.ln_f.weight, None, self._g(m.ln_f.weight), self._g(m.ln_f.bias),
            go, want_lowp=True, dropout=st.site(3 * n_layers), grad_dtype=self.grad_dtype,
        )
        del dhf
        self._notify("ln_f")

        self._pop()
        for i in reversed(range(len(self.blocks))):
            self._push(f"bwd.block{i}")
            blk, a = self.blocks[i], st.blocks[i]
            # MLP: delta = g Wp^T + bp ; dx is d(delta).  Every bias gradient of the block is the
            # column sum of the output gradient its weight-gradient GEMM streams: summed there
            self._wgrad(self._g(blk.mlp_proj.weight), dx_lp, a.g, self._g(blk.mlp_proj.bias))
            if self.fused_gemm and self.mlp_store == "gd":  # a.u holds gelu'(u): one multiply
                du = ops.linear_dx_gd(dx_lp, self._w(blk.mlp_proj.weight), a.u)
            elif self.fused_gemm:  # GELU backward in the dX GEMM's epilogue
                du = ops.linear_dx_gelu_bwd(dx_lp, self._w(blk.mlp_proj.weight), a.u)
            else:
                dg = torch.mm(dx_lp, self._w(blk.mlp_proj.weight))
                du = ops.gelu_bwd(dg, a.u, None)
                del dg
            self._wgrad(self._g(blk.mlp_fc.weight), du, a.h2, self._g(blk.mlp_fc.bias))
            wf = self._w(blk.mlp_fc.weight)
            dh2 = ops.linear_dx(du, wf) if self.fused_gemm else torch.mm(du, wf)
            del du
            # ln_2's dgamma / dbeta partial rows wait for ln_1's: one reduce launch per block
            dxm, dy_lp, ln2_parts = ops.layernorm_bwd(
                dh2, a.xm, a.mu2, a.rs2, blk.ln_2.weight, dx, self._g(blk.ln_2.weight), self._g(blk.ln_2.bias),
                None, want_lowp=True, dropout=st.site(1 + 3 * i), defer_params=True, grad_dtype=self.grad_dtype,
            )
            del dh2, dx, dx_lp
            if st.keep_col is not None:  # gradient of y * keep: padded rows feed nothing back
                dy_lp = dy_lp * st.keep_col
            # attention output projection
            self._wgrad(self._g(blk.attn.out_proj.weight), dy_lp, a.att, self._g(blk.attn.out_proj.bias))
            wo = self._w(blk.attn.out_proj.weight)
            attn_drop = st.site(2 + 3 * i)
            delta = None
            if self.fused_gemm:
                # dO plus the attention backward's row constants from one GEMM epilogue
                # (not taken -> delta None: attn_bwd computes them itself)
                datt, delta = ops.linear_dx_attn(dy_lp, wo, a.att, seqlen, head_dim=self.head_dim)
            else:
                datt = torch.mm(dy_lp, wo)
            del dy_lp
            dqkv = ops.attn_bwd(
                datt, a.qkv, a.att, a.lse, bsz, seqlen, self.n_heads, dropout=attn_drop, delta=delta,
                key_masks=st.key_masks,
            )
            del datt
            self._wgrad(self._g(blk.attn.qkv_proj.weight), dqkv, a.h1, self._g(blk.attn.qkv_proj.bias))
            wq = self._w(blk.attn.qkv_proj.weight)
            dh1 = ops.linear_dx(dqkv, wq) if self.fused_gemm else torch.mm(dqkv, wq)
            del dqkv
            dx, dx_lp, ln1_parts = ops.layernorm_bwd(
                dh1, a.xs, a.mu1, a.rs1, blk.ln_1.weight, dxm, self._g(blk.ln_1.weight), self._g(blk.ln_1.bias),
                None, want_lowp=i > 0, dropout=st.site(3 * i) if i > 0 else (0.0, 0), defer_params=True,
                grad_dtype=self.grad_dtype,
            )
            ops.ln_param_reduce(
                [ln2_parts, ln1_parts],
                [self._g(blk.ln_2.weight), self._g(blk.ln_2.bias), self._g(blk.ln_1.weight), self._g(blk.ln_1.bias)],
            )
            del dh1, dxm, ln2_parts, ln1_parts
            st.blocks[i] = None  # type: ignore[call-overload]  # free activations early
            self._notify(f"block{i}")
            self._retire_block()
            self._pop()

        ops.embedding_bwd(
            dx, st.ids, self._g(m.token_embedding.weight), self._g(m.position_embedding.weight), dropout=st.site(0)
        )
        self._notify("embed")
        self._join_side()  # clip / optimizer / loss readers on the main stream see every gradient
