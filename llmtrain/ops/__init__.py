"""Fused ops of the MI355X training path.

Each function runs the hand-written gfx950 HIP kernel (``torch.ops.llmtrain_hip.*``) when its
inputs live on a GPU and the plain-PyTorch oracle from :mod:`llmtrain.ops.reference` when they
live on the CPU (unit tests of the fused engine).  There is exactly one GPU implementation per
op and no silent fallback: a GPU tensor with the extension missing raises (``_ext.require``).
"""

from __future__ import annotations

import contextlib
import os
from collections.abc import Iterator

import torch

from llmtrain.ops import _ext
from llmtrain.ops import reference as ref

__all__ = [
    "adamw_flat",
    "add_layernorm_fwd",
    "attn_bwd",
    "attn_fwd",
    "attn_key_masks",
    "clip_coef",
    "colsum_accum",
    "cross_entropy_fwd_bwd",
    "embedding_bwd",
    "embedding_fwd",
    "gelu_bwd",
    "gelu_fwd",
    "head_dx",
    "head_logits",
    "hip_ops",
    "kernel_policy",
    "layernorm_bwd",
    "linear_dx",
    "linear_dx_gd",
    "linear_dx_gelu_bwd",
    "linear_fwd",
    "linear_fwd_gelu",
    "linear_fwd_gelu_gd",
    "ln_param_reduce",
    "policy_state",
    "restore_policy",
    "scale",
    "set_deterministic",
    "single_stream",
    "sumsq",
    "wgrad_accum",
]


def hip_ops():  # noqa: ANN201 - torch op namespace
    _ext.require()
    return torch.ops.llmtrain_hip


def _on_gpu(t: torch.Tensor) -> bool:
    return t.device.type == "cuda"


_POLICY = {"gemm_all_ours": False, "single_stream": False, "deterministic": False}

# How run.deterministic keeps the step bitwise reproducible (LLMTRAIN_DET_SCHEDULE overrides):
#  * "serial": the weight-gradient GEMMs run on the main stream (no side stream), the LM-head logits
#    and dX GEMMs on our fixed-order kernel (the logits' tuned library solution is a Stream-K kernel
#    and the one library GEMM of the configuration whose bitwise guarantee failed once,
#    profiles/r5/det/; round 6 took it off the library), and the other forward / dX GEMMs on our
#    kernel below the size cap, on hipBLASLt's tuned solutions above it.  Evidence for the library
#    GEMMs that remain: bitwise-equal repeats at micro-batch 32 of GPT-2 124M and GPT-2 XL (the
#    XL preset; 3 whole runs x 20 steps) (bench/determinism_probe.py, profiles/r4/det/,
#    profiles/r5/det/) and 800 bitwise repeats of the Stream-K solutions of the forward
#    projections, alone and beside a concurrent stream (bench/sk_repeat.py); other shapes are
#    unpinned, and each library GEMM of a serial run is named once in the log (_det_library).
#  * "ours": every forward / dX GEMM on the hand-written kernel (csrc/gemm_fused.hip), side stream
#    kept; slower because that kernel trails hipBLASLt at 128K rows (docs/round4.md).
DET_SCHEDULES = ("serial", "ours")


def set_deterministic(on: bool, schedule: str | None = None) -> bool:
    """Process-wide deterministic mode of the HIP kernels (``run.deterministic`` on GPU): the
    split-K weight-gradient GEMM and the embedding token gradient switch from float atomics to
    fixed-order reductions (every other reduction is fixed-order always), and the GEMM schedule
    becomes one of :data:`DET_SCHEDULES` — hipBLASLt's Stream-K solutions combine partial tiles in
    an order that depends on which workgroups finish first, which the weight-gradient side stream
    perturbs (bench/determinism_probe.py --runs, docs/round3.md).  Returns the previous setting.
    The CPU reference ops are deterministic anyway.  Prefer :func:`kernel_policy`, which restores
    the previous policy on exit (the Trainer scopes its steps with it)."""
    if on:
        schedule = schedule or os.environ.get("LLMTRAIN_DET_SCHEDULE", "serial")
        if schedule not in DET_SCHEDULES:
            raise ValueError(f"deterministic schedule must be one of {DET_SCHEDULES}, not {schedule!r}")
    _POLICY["gemm_all_ours"] = bool(on) and schedule == "ours"
    _POLICY["single_stream"] = bool(on) and schedule == "serial"
    _POLICY["deterministic"] = bool(on)
    if not _ext.load():
        return False
    prev = bool(torch.ops.llmtrain_hip.get_deterministic())
    torch.ops.llmtrain_hip.set_deterministic(bool(on))
    return prev


def policy_state() -> tuple[dict[str, bool], bool]:
    """Snapshot of the process-wide kernel policy: the Python routing flags and the C++
    deterministic flag (False when the extension is not loaded)."""
    cpp = bool(torch.ops.llmtrain_hip.get_deterministic()) if _ext.is_loaded() else False
    return dict(_POLICY), cpp


def restore_policy(state: tuple[dict[str, bool], bool]) -> None:
    """Undo every policy change since :func:`policy_state` returned ``state``."""
    flags, cpp = state
    _POLICY.update(flags)
    if _ext.is_loaded():
        torch.ops.llmtrain_hip.set_deterministic(bool(cpp))


@contextlib.contextmanager
def kernel_policy(deterministic: bool, schedule: str | None = None) -> Iterator[None]:
    """Run a block under ``run.deterministic = deterministic`` and restore the previous policy on
    exit, so one Trainer's setting never leaks into the next one in the same process (a test
    suite, a notebook)."""
    prev = policy_state()
    set_deterministic(deterministic, schedule)
    try:
        yield
    finally:
        restore_policy(prev)


def single_stream() -> bool:
    """True when the deterministic "serial" schedule forbids the weight-gradient side stream."""
    return _POLICY["single_stream"]


def add_layernorm_fwd(x, delta, weight, bias, eps: float, out_dtype: torch.dtype, dropout=(0.0, 0)):
    """``xs = x + dropout(delta)``, ``y = LN(xs)``; ``dropout = (p, site_seed)`` masks the branch."""
    p, seed = dropout
    if _on_gpu(x):
        xs, y, mean, rstd = hip_ops().add_layernorm_fwd(x, delta, weight, bias, eps, out_dtype, p, seed)
        return (x if delta is None else xs), y, mean, rstd
    return ref.add_layernorm_fwd(x, delta, weight, bias, eps, out_dtype, p, seed)


def layernorm_bwd(
    dy, xs, mean, rstd, weight, dresid, dweight, dbias, dy_scale=None, *, want_lowp=False, dproj_bias=None,
    dropout=(0.0, 0), defer_params=False, grad_dtype=torch.float32,
):
    """LayerNorm backward with two optional fusions for the producer of the normalised input:

    * ``want_lowp`` also returns ``dx`` in ``dy``'s dtype (the GEMM operand of the projection
      whose output was added to the residual stream), and
    * ``dproj_bias`` (fp32 ``[d]``) accumulates ``colsum(dx)`` — that projection's bias grad;

    both see the branch's dropout mask ``dropout = (p, site_seed)`` (the residual-stream ``dx``
    itself does not).  Returns ``(dx, dx_lowp | None)``.  ``grad_dtype``: storage of the
    residual-gradient stream (``dresid`` in, ``dx`` out) — fp32, or bf16 for the engine's bf16
    gradient stream, where ``dx_lowp`` without dropout IS ``dx`` (one write, not two).

    ``defer_params``: dgamma / dbeta are NOT accumulated yet; a third value ``parts`` (partial rows,
    ``[2, rows, d]``) goes to :func:`ln_param_reduce`, which reduces two LayerNorms in one launch.
    """
    p, seed = dropout
    glp = grad_dtype == torch.bfloat16
    if defer_params:
        if dproj_bias is not None:
            raise ValueError("layernorm_bwd: defer_params takes no dproj_bias")
        if _on_gpu(dy):
            dx, dx_lp, parts = hip_ops().layernorm_bwd_deferred(
                dy, xs, mean, rstd, weight, dresid, dweight, dbias, dy_scale, want_lowp, p, seed, glp
            )
            return dx, (dx_lp if want_lowp else None), parts
        pw, pb = torch.zeros_like(dweight), torch.zeros_like(dbias)
        dx = ref.layernorm_bwd(dy, xs, mean, rstd, weight, dresid, pw, pb, dy_scale, grad_dtype)
        branch = ref._apply_dropout(dx.float(), p, seed)
        return dx, (branch.to(dy.dtype) if want_lowp else None), torch.stack([pw, pb])[:, None, :]
    if _on_gpu(dy):
        dx, dx_lp = hip_ops().layernorm_bwd(
            dy, xs, mean, rstd, weight, dresid, dweight, dbias, dy_scale, want_lowp, dproj_bias, p, seed, glp
        )
        return dx, (dx_lp if want_lowp else None)
    dx = ref.layernorm_bwd(dy, xs, mean, rstd, weight, dresid, dweight, dbias, dy_scale, grad_dtype)
    branch = ref._apply_dropout(dx.float(), p, seed)
    if dproj_bias is not None:
        ref.colsum_accum(branch, dproj_bias)
    return dx, (branch.to(dy.dtype) if want_lowp else None)


def ln_param_reduce(parts: list, dst: list) -> None:
    """``dst[2i] += rows of parts[i][0]``, ``dst[2i + 1] += rows of parts[i][1]`` for the deferred
    LayerNorm backwards of :func:`layernorm_bwd` — one fixed-order launch on GPU for LayerNorms with
    equal partial-row counts (a block's ln_2 and ln_1), separate launches otherwise."""
    if not parts:
        return
    if parts[0].device.type != "cuda":
        for i, pr in enumerate(parts):
            dst[2 * i] += pr[0].sum(0)
            dst[2 * i + 1] += pr[1].sum(0)
        return
    if len({tuple(pr.shape) for pr in parts}) == 1:
        hip_ops().ln_param_reduce(list(parts), list(dst))
        return
    for i, pr in enumerate(parts):
        hip_ops().ln_param_reduce([pr], [dst[2 * i], dst[2 * i + 1]])


def cross_entropy_fwd_bwd(logits, labels, vocab: int, row_weight):
    if _on_gpu(logits):
        return hip_ops().cross_entropy_fwd_bwd(logits, labels, vocab, row_weight)
    return ref.cross_entropy_fwd_bwd(logits, labels, vocab, row_weight)


def scale(x, s):
    """``x * s`` for a 0-/1-element fp32 device scalar ``s`` (an autograd upstream gradient):
    one HIP pass with fp32 math and a single rounding on GPU, no host sync."""
    if _on_gpu(x) and x.is_contiguous() and x.numel() % 8 == 0 and x.dtype in (torch.bfloat16, torch.float32):
        return hip_ops().scale(x, s.reshape(1).float())
    return (x.float() * s.float()).to(x.dtype)


def gelu_fwd(u):
    if _on_gpu(u):
        return hip_ops().gelu_fwd(u)
    return ref.gelu_fwd(u)


def gelu_bwd(dg, u, dbias):
    if _on_gpu(dg):
        return hip_ops().gelu_bwd(dg, u, dbias)
    return ref.gelu_bwd(dg, u, dbias)


def colsum_accum(dy, out) -> None:
    if _on_gpu(dy):
        hip_ops().colsum_accum(dy, out)
    else:
        ref.colsum_accum(dy, out)


def embedding_fwd(ids, wte, wpe, dropout=(0.0, 0), out_dtype=torch.float32):
    """Token + position embedding (+ dropout), ``out_dtype`` = the residual stream's storage."""
    p, seed = dropout
    if _on_gpu(ids):
        return hip_ops().embedding_fwd(ids, wte, wpe, p, seed, out_dtype == torch.bfloat16)
    return ref.embedding_fwd(ids, wte, wpe, p, seed, out_dtype)


def embedding_bwd(dx, ids, dwte, dwpe, dropout=(0.0, 0)) -> None:
    """Token / position embedding gradients from the residual-stream gradient ``dx`` (fp32 or
    bf16: the scatter kernels read either stream as is)."""
    p, seed = dropout
    if _on_gpu(dx):
        hip_ops().embedding_bwd(dx.contiguous(), ids, dwte, dwpe, p, seed)
    else:
        ref.embedding_bwd(dx, ids, dwte, dwpe, p, seed)


def attn_key_masks(mask: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Device forms of a ``[B, T]`` key-padding mask for the attention kernels: ``key_bits``
    ``[B, ceil(T/64)]`` int64 (bit j of word w = key 64w + j is valid; the forward reads one word
    per 64-key tile) and ``key_valid`` ``[B, T]`` uint8 (the backward reads its lane's key)."""
    bsz, seqlen = mask.shape
    valid = mask.bool()
    words = -(-seqlen // 64)
    padded = torch.zeros(bsz, words * 64, dtype=torch.int64, device=mask.device)
    padded[:, :seqlen] = valid.to(torch.int64)
    shifts = torch.arange(64, dtype=torch.int64, device=mask.device)
    bits = (padded.view(bsz, words, 64) << shifts).sum(dim=-1)  # wraps into bit 63 as int64
    return bits.contiguous(), valid.to(torch.uint8).contiguous()


def attn_fwd(qkv, bsz: int, seqlen: int, n_heads: int, dropout=(0.0, 0), key_masks=None):
    """Causal flash attention over packed ``qkv``; ``key_masks`` = :func:`attn_key_masks` of the
    batch's key-padding mask (None = every key valid)."""
    p, seed = dropout
    if _on_gpu(qkv):
        bits = None if key_masks is None else key_masks[0]
        return hip_ops().attn_fwd(qkv, bsz, seqlen, n_heads, p, seed, bits)
    valid = None if key_masks is None else key_masks[1]
    return ref.attn_fwd(qkv, bsz, seqlen, n_heads, p, seed, valid)


def attn_bwd(
    dout, qkv, out, lse, bsz: int, seqlen: int, n_heads: int, dropout=(0.0, 0), qkv_bias_grad=None, delta=None,
    key_masks=None,
):
    """Attention backward -> packed ``dqkv``; ``qkv_bias_grad`` (fp32 ``[3d]``), when given,
    accumulates ``colsum(dqkv)`` (fused into the kernels on GPU).  ``delta`` (GPU): the row
    constants ``rowsum(dO * O)`` already computed by :func:`linear_dx_attn`, which then also added
    the V part of ``qkv_bias_grad`` when there is no dropout; the delta pass is skipped."""
    p, seed = dropout
    valid = None if key_masks is None else key_masks[1]
    if _on_gpu(dout):
        return hip_ops().attn_bwd(dout, qkv, out, lse, bsz, seqlen, n_heads, p, seed, qkv_bias_grad, delta, valid)
    dqkv = ref.attn_bwd(dout, qkv, out, lse, bsz, seqlen, n_heads, p, seed, valid)
    if qkv_bias_grad is not None:
        ref.colsum_accum(dqkv, qkv_bias_grad)
    return dqkv


# Where the fused GEMM pays in a real step (same-box A/B, docs/performance.md): GPT-2 XL micro-batch
# 16 (A operands 52 MB) +3 %; GPT-2 124M at 64K-128K tokens per step (A 100-600 MB) -1.4 % although
# each GEMM alone is ahead of hipBLASLt at 64K: its persistent, statically scheduled 160 KiB-LDS
# workgroups start late on CUs still draining the previous kernel.  Above this many A bytes the
# engine stays on hipBLASLt.
FGEMM_MAX_A_BYTES = int(float(os.environ.get("LLMTRAIN_FGEMM_MAX_A_MB", "64")) * 2**20)  # A/B knob
# Ops that stay on the library GEMM at every size (outside deterministic mode's "ours" schedule)
FGEMM_NEVER = frozenset(t for t in os.environ.get("LLMTRAIN_FGEMM_NEVER", "").split(",") if t)
# Ops that take the fused GEMM at any A size.  dx_gelu: the MLP-projection dX with GELU backward +
# fc-bias grad in the epilogue replaces a hipBLASLt GEMM plus a full [M, 4d] read-modify pass, and
# wins in the whole 124M step (same-box, micro-batch 128: +0.9 %, 994.9k/995.5k vs 985.8k/986.8k
# tok/s).  dx_attn: the attention out-projection dX with the backward's delta rows and the V-bias
# column sums in the epilogue (deletes the delta pass; same-box mb 128: 1,076.3k vs 1,074.5k tok/s,
# profiles/r3/ab_dx_attn_any_size_mb128.txt).  Adding the plain dX GEMMs (-0.4 %) or the forward
# GEMMs (-1.6 %) at this size loses: hipBLASLt's 256x256 kernels run 1.1-1.3 PF on these shapes
# against 0.86-1.14 PF for ours (profiles/r3/fgemm_wide_v2_ab_m131k.log).  With non-temporal output
# stores at this size, fc + bias + GELU on ours beats hipBLASLt + the GELU pass alone (0.725 vs
# 0.808 ms) but runs 0.86 ms per call inside the step and the step loses 0.4-1.0 % (qkv forward
# too: -1.2 %; profiles/r3/nt/), so those stay on hipBLASLt.
FGEMM_ANY_SIZE = frozenset(os.environ.get("LLMTRAIN_FGEMM_ANY", "dx_gelu,dx_attn").split(","))  # A/B knob


_WARNED: set[str] = set()


def _det_fallback(what: str, always: bool = False) -> None:
    """A GEMM of a deterministic run that cannot take the hand-written fixed-order kernel (its
    shape or alignment is outside what csrc/gemm_fused.hip takes: K % 64 == 0, K >= 256, N % 8 ==
    0, 16-byte aligned operands) runs on hipBLASLt instead, whose split / Stream-K solutions may
    combine partial sums in completion order.  In the "ours" schedule (every GEMM promised on our
    kernel), and for the GEMMs the serial schedule keeps off the library (``always``), that breaks
    the promise: say so once per distinct case instead of failing silently."""
    if (_POLICY["gemm_all_ours"] or (always and _POLICY["deterministic"])) and what not in _WARNED:
        _WARNED.add(what)
        import warnings

        warnings.warn(
            f"run.deterministic: {what} cannot take the fixed-order GEMM kernel and runs on hipBLASLt "
            "(bitwise run-to-run reproducibility of this GEMM is not guaranteed)", RuntimeWarning, stacklevel=3,
        )


def _det_library(what: str) -> None:
    """Serial deterministic schedule: ``what`` runs on a tuned hipBLASLt solution by design.  Those
    were bitwise reproducible in every repeat measured (GPT-2 124M at micro-batch 8 and 32, GPT-2 XL
    at 32; profiles/r4/det/, profiles/r5/det/), which pins no other shape: name each such GEMM once
    in the log, so a run on a
    new shape knows which of its GEMMs rest on that evidence (LLMTRAIN_DET_SCHEDULE=ours moves every
    one the kernel can take onto the fixed-order kernel)."""
    if _POLICY["single_stream"] and what not in _WARNED:
        _WARNED.add(what)
        import logging

        logging.getLogger(__name__).warning(
            "run.deterministic (serial schedule): %s runs on hipBLASLt; its reproducibility is measured "
            "for GPT-2 124M at micro-batch 8/32 and GPT-2 XL at 32 only", what,
        )


def _lib_mm(a: torch.Tensor, b_t: torch.Tensor, bias: torch.Tensor | None = None, *, op: str) -> torch.Tensor:
    """``a @ b_t (+ bias)`` on the library GEMM, logged once per shape in the serial schedule."""
    if _POLICY["single_stream"] and a.is_cuda:
        _det_library(f"GEMM {op} M={a.shape[0]} K={a.shape[1]} N={b_t.shape[1]}")
    return torch.mm(a, b_t) if bias is None else torch.addmm(bias, a, b_t)


def _fgemm_ok(a: torch.Tensor, k: int, n: int, *others: torch.Tensor | None, op: str = "") -> bool:
    """Shapes/placements the fused MFMA GEMM (csrc/gemm_fused.hip) takes and wins on:
    K % 64 == 0, K >= 256, N % 8 == 0, 16-byte aligned operands, A small enough (see above)."""
    if not (k % 64 == 0 and k >= 256 and n % 8 == 0):
        _det_fallback(f"GEMM {op or 'linear'} K={k} N={n} (needs K % 64 == 0, K >= 256, N % 8 == 0)")
        return False
    if a.numel() * a.element_size() > FGEMM_MAX_A_BYTES and op not in FGEMM_ANY_SIZE and not _POLICY["gemm_all_ours"]:
        return False
    if op in FGEMM_NEVER and not _POLICY["gemm_all_ours"]:
        return False
    if not all(t is None or t.data_ptr() % 16 == 0 for t in (a, *others)):
        _det_fallback(f"GEMM {op or 'linear'} with an operand not 16-byte aligned")
        return False
    return True


def _fgemm_ok_any_size(a: torch.Tensor, k: int, n: int, *others: torch.Tensor | None, op: str = "") -> bool:
    """:func:`_fgemm_ok` without the A-size routing cap (row-chunked callers: the LM head)."""
    if not (k % 64 == 0 and k >= 256 and n % 8 == 0):
        _det_fallback(f"GEMM {op or 'linear'} K={k} N={n} (needs K % 64 == 0, K >= 256, N % 8 == 0)", always=True)
        return False
    if not all(t is None or t.data_ptr() % 16 == 0 for t in (a, *others)) or a.stride(1) != 1:
        _det_fallback(f"GEMM {op or 'linear'} with an operand not 16-byte aligned", always=True)
        return False
    return True


# The hand-written GEMM's buffer descriptors and tile offsets are 32-bit byte offsets: every [M, K]
# operand and [M, N] output must stay below 2 GiB (the binding refuses larger ones).  Larger GEMMs run
# as row chunks (GPT-2 124M at micro-batch >= ~342, XL's d_ff = 6400 past ~168K rows), each chunk a
# whole number of sequences for epilogue 3.
_OFFSET_LIMIT = 2**31


def _gemm_rows(a, b, b_kn: bool, epilogue: int, bias=None, u=None, dbias=None, seq_len: int = 0):
    """``hip_ops().gemm_fused`` over row chunks small enough for its 32-bit offsets."""
    m, k = a.shape
    n = b.shape[1] if b_kn else b.shape[0]
    align = 256 * seq_len if epilogue == 3 else 256
    rows = max(align, (_OFFSET_LIMIT - 1) // (2 * max(k, n)) // align * align)
    extra = () if epilogue < 3 else (seq_len,)
    if m <= rows:
        return tuple(hip_ops().gemm_fused(a, b, b_kn, epilogue, bias, u, dbias, *extra))
    parts = [
        hip_ops().gemm_fused(a[r0 : r0 + rows], b, b_kn, epilogue, bias,
                             None if u is None else u[r0 : r0 + rows], dbias, *extra)
        for r0 in range(0, m, rows)
    ]
    out = torch.cat([p[0] for p in parts])
    if parts[0][1] is None:
        return out, None
    return out, torch.cat([p[1] for p in parts])


_TUNED_BIAS_GEMMS: set[tuple[int, int, int]] | None = None


def _library_tuned_bias_gemm(m: int, n: int, k: int) -> bool:
    """Whether the shipped TunableOp table (llmtrain/runtime/tuned/) holds a measured library
    solution for the bias GEMM ``[m, k] @ [n, k]^T + bias``: such shapes were timed against our
    kernel when the table was made (micro-batch 32: qkv 0.109 vs 0.116 ms, out 0.041 vs 0.053 ms,
    profiles/r4/mb32/) and stay on the library."""
    global _TUNED_BIAS_GEMMS
    if _TUNED_BIAS_GEMMS is None:
        from ..runtime.tuning import TUNED_TABLE, tuned_gemms_active

        if not tuned_gemms_active():  # not (yet) loaded in this process: nothing is routed by it
            return False
        shapes: set[tuple[int, int, int]] = set()
        if TUNED_TABLE.is_file():
            for line in TUNED_TABLE.read_text().splitlines():
                parts = line.split(",")
                if len(parts) >= 2 and parts[0] == "GemmAndBiasTunableOp_BFloat16_TN" and parts[1].startswith("tn_"):
                    dims = parts[1].split("_")
                    shapes.add((int(dims[2]), int(dims[1]), int(dims[3])))  # tn_{N}_{M}_{K}: (M, N, K)
        _TUNED_BIAS_GEMMS = shapes
    return (m, n, k) in _TUNED_BIAS_GEMMS


def linear_fwd(x, w, bias=None):
    """``x @ w^T + bias`` (nn.Linear forward, bf16 out).  GPU: the fused MFMA GEMM with the bias in
    its epilogue where the shape allows and the library has no measured solution for it, else
    hipBLASLt."""
    if (_on_gpu(x) and x.dtype == torch.bfloat16 and _fgemm_ok(x, x.shape[1], w.shape[0], w, bias, op="fwd")
            and (_POLICY["deterministic"] or bias is None
                 or not _library_tuned_bias_gemm(x.shape[0], w.shape[0], x.shape[1]))):
        return _gemm_rows(x, w, False, 0, bias)[0]
    return _lib_mm(x, w.t(), bias, op="fwd")


def linear_fwd_gelu(x, w, bias=None):
    """``u = x @ w^T + bias`` and ``g = gelu(u)`` (exact erf GELU of the bf16 ``u``, which the
    backward reads): on GPU the GELU rides in the GEMM epilogue, no separate pass over ``u``."""
    if _on_gpu(x) and x.dtype == torch.bfloat16 and _fgemm_ok(x, x.shape[1], w.shape[0], w, bias, op="fwd_gelu"):
        u, g = _gemm_rows(x, w, False, 1, bias)
        return u, g
    u = _lib_mm(x, w.t(), bias, op="fc fwd")
    return u, gelu_fwd(u)


def linear_fwd_gelu_gd(x, w, bias=None):
    """``gd = gelu'(u)`` and ``g = gelu(u)`` of ``u = x @ w^T + bias`` (the bf16 ``u``, as the
    backward would read it): the fc forward keeps the GELU derivative instead of the
    pre-activation, so the MLP-projection dX epilogue (:func:`linear_dx_gd`) multiplies by a stored
    value instead of evaluating erf per element.  GPU: one fused-GEMM epilogue (4) at any size;
    shapes that kernel does not take form ``u`` on the library and the two maps with torch ops."""
    if (_on_gpu(x) and x.dtype == torch.bfloat16 and _fgemm_ok_any_size(x, x.shape[1], w.shape[0], w, bias,
                                                                     op="fc fwd + GELU'")):
        gd, g = _gemm_rows(x, w, False, 4, bias)
        return gd, g
    u = _lib_mm(x, w.t(), bias, op="fc fwd") if _on_gpu(x) else (
        torch.mm(x, w.t()) if bias is None else torch.addmm(bias, x, w.t()))
    return ref.gelu_grad(u), gelu_fwd(u)


def linear_dx_gd(dy, w, gd, dbias=None):
    """``du = (dy @ w) * gd`` and ``dbias += colsum(du)`` with ``gd = gelu'(u)`` stored by
    :func:`linear_fwd_gelu_gd`: the MLP-projection data gradient and the GELU backward in one GEMM
    epilogue (5) on GPU."""
    if _on_gpu(dy) and dy.dtype == torch.bfloat16 and _fgemm_ok_any_size(dy, dy.shape[1], w.shape[1], w, gd,
                                                                         op="MLP-projection dX * gelu'"):
        return _gemm_rows(dy, w, True, 5, None, gd, dbias)[0]
    dg = _lib_mm(dy, w, op="MLP-projection dX") if _on_gpu(dy) else torch.mm(dy, w)
    du = (dg.float() * gd.float()).to(dy.dtype)
    if dbias is not None:
        colsum_accum(du, dbias)
    return du


def linear_dx(dy, w):
    """``dy @ w`` (data gradient of nn.Linear with weight ``w [out, in]``)."""
    if _on_gpu(dy) and dy.dtype == torch.bfloat16 and _fgemm_ok(dy, dy.shape[1], w.shape[1], w, op="dx"):
        return _gemm_rows(dy, w, True, 0)[0]
    return _lib_mm(dy, w, op="dX")


# rows per launch of the LM-head GEMMs on the hand-written kernel: its buffer descriptors take
# 32-bit byte offsets, and [rows, 50304] bf16 must stay below 2 GiB
_HEAD_ROWS = 16384


def head_logits(h, w):
    """``logits = h @ w^T`` for the vocab-padded LM head ``w [Vp, d]``: hipBLASLt on the fast path;
    in deterministic mode (either schedule) row chunks of the hand-written fixed-order kernel,
    written in place into one ``[M, Vp]`` output.  The library's tuned solution for this shape is a
    Stream-K kernel (``SK3``), which combines partial tiles in completion order — the one library
    GEMM left in the serial schedule when its bitwise guarantee failed once
    (profiles/r5/det/pytest_gpu_serial_divergence.txt, docs/round6.md §2)."""
    if not (_on_gpu(h) and _POLICY["deterministic"] and h.dtype == torch.bfloat16
            and _fgemm_ok_any_size(h, h.shape[1], w.shape[0], w, op="LM-head logits")):
        return _lib_mm(h, w.t(), op="LM-head logits")
    out = torch.empty(h.shape[0], w.shape[0], dtype=h.dtype, device=h.device)
    for r0 in range(0, h.shape[0], _HEAD_ROWS):
        r1 = min(h.shape[0], r0 + _HEAD_ROWS)
        hip_ops().gemm_fused(h[r0:r1], w, False, 0, None, None, None, 0, out[r0:r1])
    return out


def head_dx(dlogits, w):
    """``dh = dlogits @ w`` (LM-head data gradient, ``w [Vp, d]``), row-chunked like
    :func:`head_logits` on our kernel.  Deterministic mode always takes our kernel here: this is the
    step's only GEMM with a 50304-deep reduction, where the library picks split / Stream-K
    solutions whose partial sums combine in completion order — the one run-to-run difference left
    in the serial schedule (bench/determinism_probe.py at micro-batch 8: the gradients first differ
    at ln_f, the head dX's output)."""
    k, n = dlogits.shape[1], w.shape[1]
    if not (_on_gpu(dlogits) and _POLICY["deterministic"] and dlogits.dtype == torch.bfloat16
            and k % 64 == 0 and k >= 256 and n % 8 == 0  # the size cap does not apply: row chunks
            and dlogits.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0 and dlogits.stride(1) == 1):
        if _on_gpu(dlogits) and _POLICY["deterministic"]:
            _det_fallback(f"LM-head dX K={k} N={n}", always=True)
        return torch.mm(dlogits, w)
    out = torch.empty(dlogits.shape[0], w.shape[1], dtype=dlogits.dtype, device=dlogits.device)
    for r0 in range(0, dlogits.shape[0], _HEAD_ROWS):
        r1 = min(dlogits.shape[0], r0 + _HEAD_ROWS)
        hip_ops().gemm_fused(dlogits[r0:r1], w, True, 0, None, None, None, 0, out[r0:r1])
    return out


def linear_dx_gelu_bwd(dy, w, u, dbias=None):
    """``du = (dy @ w) * gelu'(u)`` and ``dbias += colsum(du)``: the data gradient of the MLP
    projection fused with the GELU backward and the fc bias gradient (one GEMM epilogue on GPU
    instead of a GEMM plus a full read-modify pass over the [M, d_ff] activations)."""
    if _on_gpu(dy) and dy.dtype == torch.bfloat16 and _fgemm_ok(dy, dy.shape[1], w.shape[1], w, u, op="dx_gelu"):
        return _gemm_rows(dy, w, True, 2, None, u, dbias)[0]
    return gelu_bwd(_lib_mm(dy, w, op="MLP-projection dX"), u, dbias)


def linear_dx_attn(dy, w, att, seqlen: int, v_bias_grad=None, head_dim: int = 64):
    """Data gradient of the attention output projection, ``dO = dy @ w``, plus the flash-attention
    backward's row constants ``delta[b, h, t] = sum_d dO * O`` (``att`` = the attention output O)
    and, when given, ``v_bias_grad += colsum(dO)`` (the V part of the qkv bias gradient, valid
    without attention dropout).  GPU: one fused GEMM epilogue (csrc/gemm_fused.hip, epilogue 3)
    replacing the separate pass that re-read dO and O.  Returns ``(dO, delta)``; ``delta`` is None
    when the GEMM is not taken (the attention backward then computes it itself, and the caller
    must leave ``v_bias_grad`` to it)."""
    if (
        _on_gpu(dy)
        and dy.dtype == torch.bfloat16
        and head_dim == 64  # the epilogue's per-head row dots are 64 columns wide
        and dy.shape[0] % seqlen == 0
        and w.shape[1] % 64 == 0
        and _fgemm_ok(dy, dy.shape[1], w.shape[1], w, att, op="dx_attn")
    ):
        return _gemm_rows(dy, w, True, 3, None, att, v_bias_grad, seqlen)
    if _on_gpu(dy) and head_dim != 64:
        # the epilogue's row dots need 64-wide heads: a plain dX GEMM (fixed-order kernel where the
        # shape allows, e.g. the reference presets' d = 256 / 384) and attn_bwd forms delta itself
        return linear_dx(dy, w), None
    return _lib_mm(dy, w, op="attention out-projection dX"), None


def wgrad_accum(dst, dy, x, *, bias=None) -> None:
    """``dst (fp32 [N, K]) += dy[M, N]^T @ x[M, K]`` and, with ``bias`` (fp32 ``[N]``),
    ``bias += colsum(dy)`` — the weight and bias gradients of an nn.Linear whose output gradient
    is ``dy`` (``dy`` may be a column slice with a larger row stride).  GPU: the split-K MFMA GEMM
    of csrc/gemm_wgrad_pp.hip with the bias column sums fused."""
    if _on_gpu(dst):
        hip_ops().wgrad_gemm_pp(dy, x, dst, bias, 0, -1)
        return
    dst.addmm_(dy.t().float(), x.float())
    if bias is not None:
        colsum_accum(dy, bias)


def sumsq(x):
    if _on_gpu(x):
        return hip_ops().sumsq(x)
    return ref.sumsq(x)


def clip_coef(sumsq_t, max_norm: float):
    """``[norm, coef]`` of the gradient clip from the global squared norm (fp32, one element):
    ``norm = sqrt(sumsq)``, ``coef = min(1, max_norm / (norm + 1e-6))`` (``clip_grad_norm_``), and
    ``coef = NaN`` when the norm is NaN/Inf, which makes :func:`adamw_flat` skip the step."""
    if _on_gpu(sumsq_t):
        return hip_ops().clip_coef(sumsq_t.reshape(1).float(), float(max_norm))
    return ref.clip_coef(sumsq_t, max_norm)


def adamw_flat(
    param, grad, exp_avg, exp_avg_sq, shadow, *, lr, beta1, beta2, eps, weight_decay, step, grad_scale, dyn=None,
    skipped=None,
):
    """``dyn`` (GPU only): device ``[decay, step_size, bc2_sqrt]`` read by the kernel instead of the
    values formed from ``lr``/``step`` — a hipGraph-captured step stages them before each replay.
    A non-finite ``grad_scale`` skips the update (nothing is written); ``skipped`` (int32 ``[2]``,
    optional) then counts it: ``[total, consecutive]``, the second reset by an applied step."""
    if _on_gpu(param):
        hip_ops().adamw_flat(
            param, grad, exp_avg, exp_avg_sq, shadow, lr, beta1, beta2, eps, weight_decay, step, grad_scale, dyn,
            skipped,
        )
        return
    if dyn is not None:
        raise ValueError("adamw_flat: device-staged scalars exist only on the GPU path")
    ref.adamw_flat(
        param, grad, exp_avg, exp_avg_sq, shadow, lr=lr, beta1=beta1, beta2=beta2, eps=eps,
        weight_decay=weight_decay, step=step, grad_scale=grad_scale, skipped=skipped,
    )
