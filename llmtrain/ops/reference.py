"""Plain-PyTorch fp32 reference implementations of every fused op.

These are the numerics oracles for the HIP kernels (``tests/test_kernels_gpu.py`` compares each
kernel against the function of the same name here) and the implementation used when the fused
GPT engine runs on CPU (unit tests of the hand-written backward).  Signatures mirror the HIP
ops in ``csrc/bindings.cpp`` exactly, including in-place accumulation into gradient buffers.

Layout conventions shared with the kernels:
* activations are row-major ``[M, C]`` with ``M = B*T`` tokens;
* ``qkv`` is the packed projection output ``[B, T, 3, H, Dh]`` (viewed as ``[B*T, 3*d]``);
* attention ``lse`` is the natural-log softmax normaliser per (b, h, t), ``[B, H, T]`` fp32;
* weight/bias gradient buffers are fp32 and are *accumulated into* (never overwritten).
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F

__all__ = [
    "adamw_flat",
    "clip_coef",
    "dropout_keep",
    "dropout_params",
    "dropout_site_seed",
    "add_layernorm_fwd",
    "attn_bwd",
    "attn_fwd",
    "colsum_accum",
    "cross_entropy_fwd_bwd",
    "embedding_bwd",
    "embedding_fwd",
    "gelu_bwd",
    "gelu_grad",
    "gelu_fwd",
    "layernorm_bwd",
    "sumsq",
]

_INV_SQRT2 = 1.0 / math.sqrt(2.0)
_INV_SQRT_2PI = 1.0 / math.sqrt(2.0 * math.pi)
_M32 = 0xFFFFFFFF


# ---- dropout masks (bit-identical to csrc/common.h drop_keep) --------------------------------


def _mix32(x: torch.Tensor) -> torch.Tensor:
    """lowbias32 on int64 tensors holding uint32 values (products wrap mod 2^64; low 32 bits exact)."""
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    return x ^ (x >> 16)


def mix32_int(x: int) -> int:
    """Scalar lowbias32 (host-side seed derivation)."""
    x &= _M32
    x ^= x >> 16
    x = (x * 0x7FEB352D) & _M32
    x ^= x >> 15
    x = (x * 0x846CA68B) & _M32
    return x ^ (x >> 16)


def dropout_site_seed(step_seed: int, site: int) -> int:
    """Seed of one dropout site (one tensor of one layer) for one forward pass."""
    return mix32_int((step_seed & _M32) ^ ((site * 0x9E3779B9) & _M32))


def dropout_params(p: float) -> tuple[int, float]:
    """``(thr, scale)`` exactly as the HIP side derives them (thr = round(p * 2^16))."""
    thr = min(int(round(p * 65536.0)), 65535) if p > 0 else 0
    return thr, (65536.0 / (65536 - thr) if thr else 1.0)


def dropout_keep(seed: int, thr: int, idx: torch.Tensor) -> torch.Tensor:
    """Keep-mask for element indices ``idx`` (int64) of a site with ``seed``."""
    if thr == 0:
        return torch.ones_like(idx, dtype=torch.bool)
    pair = idx >> 1
    h = _mix32((pair & _M32) ^ (seed & _M32) ^ (((pair >> 32) * 0x85EBCA6B) & _M32))
    half = torch.where((idx & 1).bool(), h >> 16, h & 0xFFFF)
    return half >= thr


def _apply_dropout(x: torch.Tensor, p: float, seed: int) -> torch.Tensor:
    """Mask a row-major tensor whose element ``i`` (flat index) belongs to the site."""
    thr, scale = dropout_params(p)
    if thr == 0:
        return x
    idx = torch.arange(x.numel(), device=x.device, dtype=torch.int64).view(x.shape)
    return torch.where(dropout_keep(seed, thr, idx), x * scale, torch.zeros_like(x))


def attn_dropout_keep(seed: int, p: float, bsz: int, n_heads: int, seqlen: int, device) -> torch.Tensor:
    """``[B, H, T, T]`` keep-mask of attention probabilities (plane seed per (b, h), index q*T+k)."""
    thr, _ = dropout_params(p)
    bh = torch.arange(bsz * n_heads, dtype=torch.int64, device=device)
    pseed = _mix32((seed + bh * 0x9E3779B9) & _M32).view(bsz, n_heads, 1, 1)
    e = torch.arange(seqlen * seqlen, dtype=torch.int64, device=device).view(1, 1, seqlen, seqlen)
    pair = e >> 1
    h = _mix32((pair ^ pseed) & _M32)
    half = torch.where((e & 1).bool(), h >> 16, h & 0xFFFF)
    return half >= thr


def add_layernorm_fwd(
    x: torch.Tensor,
    delta: torch.Tensor | None,
    weight: torch.Tensor,
    bias: torch.Tensor,
    eps: float,
    out_dtype: torch.dtype,
    dropout_p: float = 0.0,
    dropout_seed: int = 0,
) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """``xs = x + dropout(delta)`` (fp32 add), ``y = LN(xs)`` cast to ``out_dtype``.

    Returns ``(xs, y, mean, rstd)``; when ``delta`` is None ``xs`` is ``x`` itself.  A bf16 ``x``
    (the engine's bf16 residual stream) gives a bf16 ``xs``, and the statistics are those of the
    rounded ``xs`` (as the HIP kernel computes them).
    """
    xs = x if delta is None else (x.float() + _apply_dropout(delta.float(), dropout_p, dropout_seed)).to(x.dtype)
    xs32 = xs.float()
    mean = xs32.mean(dim=-1)
    var = (xs32 - mean[:, None]).pow(2).mean(dim=-1)
    rstd = torch.rsqrt(var + eps)
    y = (xs32 - mean[:, None]) * rstd[:, None] * weight.float() + bias.float()
    return xs, y.to(out_dtype), mean, rstd


def layernorm_bwd(
    dy: torch.Tensor,
    xs: torch.Tensor,
    mean: torch.Tensor,
    rstd: torch.Tensor,
    weight: torch.Tensor,
    dresid: torch.Tensor | None,
    dweight: torch.Tensor,
    dbias: torch.Tensor,
    dy_scale: torch.Tensor | None = None,
    grad_dtype: torch.dtype = torch.float32,
) -> torch.Tensor:
    """LayerNorm backward. Returns ``dx`` = ``dresid + dLN/dx`` (fp32 math, stored as
    ``grad_dtype``: bf16 for the engine's bf16 gradient stream); accumulates dγ, dβ.

    ``dy_scale`` (0-d fp32 tensor) multiplies ``dy`` first (used to fold the loss gradient
    scale into the first backward kernel without a host sync).
    """
    g = dy.float()
    if dy_scale is not None:
        g = g * dy_scale.float()
    xhat = (xs.float() - mean[:, None]) * rstd[:, None]
    dweight += (g * xhat).sum(dim=0)
    dbias += g.sum(dim=0)
    gw = g * weight.float()
    dx = rstd[:, None] * (gw - gw.mean(dim=-1, keepdim=True) - xhat * (gw * xhat).mean(dim=-1, keepdim=True))
    if dresid is not None:
        dx = dx + dresid.float()
    return dx.to(grad_dtype)


def cross_entropy_fwd_bwd(
    logits: torch.Tensor, labels: torch.Tensor, vocab: int, row_weight: torch.Tensor
) -> torch.Tensor:
    """Per-row CE loss over the first ``vocab`` columns; overwrites ``logits`` with dlogits.

    ``logits`` ``[M, Vp]`` (``Vp >= vocab``, padded columns ignored and given zero gradient),
    ``labels`` ``[M]`` int64 (negative = ignored row: loss 0, gradient 0), ``row_weight`` ``[M]``
    fp32 — the gradient of row ``i`` is ``(softmax - onehot) * row_weight[i]``.
    Returns the unweighted per-row loss ``[M]`` fp32.
    """
    z = logits[:, :vocab].float()
    lse = torch.logsumexp(z, dim=-1)
    valid = labels >= 0
    safe = torch.where(valid, labels, torch.zeros_like(labels))
    picked = z.gather(1, safe[:, None]).squeeze(1)
    loss = torch.where(valid, lse - picked, torch.zeros_like(lse))
    grad = torch.softmax(z, dim=-1)
    grad[torch.arange(z.shape[0], device=z.device), safe] -= 1.0
    grad = grad * (row_weight * valid.float())[:, None]
    logits[:, :vocab] = grad.to(logits.dtype)
    if logits.shape[1] > vocab:
        logits[:, vocab:] = 0
    return loss


def gelu_fwd(u: torch.Tensor) -> torch.Tensor:
    """Exact (erf) GELU, same dtype as the input (``nn.GELU()`` default, reference gpt.py:95)."""
    return F.gelu(u.float()).to(u.dtype)


def gelu_bwd(dg: torch.Tensor, u: torch.Tensor, dbias: torch.Tensor | None) -> torch.Tensor:
    """``du = dg * gelu'(u)`` in ``u.dtype``; accumulates ``colsum(du)`` into ``dbias``."""
    uf = u.float()
    cdf = 0.5 * (1.0 + torch.erf(uf * _INV_SQRT2))
    pdf = torch.exp(-0.5 * uf * uf) * _INV_SQRT_2PI
    du = dg.float() * (cdf + uf * pdf)
    if dbias is not None:
        dbias += du.sum(dim=0)
    return du.to(u.dtype)


def gelu_grad(u: torch.Tensor) -> torch.Tensor:
    """``gelu'(u)`` of the exact (erf) GELU, in ``u.dtype`` (computed in fp32)."""
    uf = u.float()
    cdf = 0.5 * (1.0 + torch.erf(uf * _INV_SQRT2))
    pdf = torch.exp(-0.5 * uf * uf) * _INV_SQRT_2PI
    return (cdf + uf * pdf).to(u.dtype)


def colsum_accum(dy: torch.Tensor, out: torch.Tensor) -> None:
    """``out += dy.sum(0)`` in fp32 (bias gradients)."""
    out += dy.float().sum(dim=0)


def embedding_fwd(
    ids: torch.Tensor, wte: torch.Tensor, wpe: torch.Tensor, dropout_p: float = 0.0, dropout_seed: int = 0,
    out_dtype: torch.dtype = torch.float32,
) -> torch.Tensor:
    """``x[b*T+t] = dropout(wte[ids[b,t]] + wpe[t])`` → ``[B*T, d]`` (fp32 math, ``out_dtype``)."""
    bsz, seqlen = ids.shape
    x = wte.float()[ids.reshape(-1)] + wpe.float()[:seqlen].repeat(bsz, 1)
    return _apply_dropout(x, dropout_p, dropout_seed).to(out_dtype)


def embedding_bwd(
    dx: torch.Tensor,
    ids: torch.Tensor,
    dwte: torch.Tensor,
    dwpe: torch.Tensor,
    dropout_p: float = 0.0,
    dropout_seed: int = 0,
) -> None:
    """Scatter-add (masked) token gradients into ``dwte``; sum over the batch into ``dwpe[:T]``."""
    bsz, seqlen = ids.shape
    dx = _apply_dropout(dx.float(), dropout_p, dropout_seed)
    dwte.index_add_(0, ids.reshape(-1), dx.float())
    dwpe[:seqlen] += dx.float().view(bsz, seqlen, -1).sum(dim=0)


def _split_qkv(qkv: torch.Tensor, bsz: int, seqlen: int, n_heads: int):
    d = qkv.shape[-1] // 3
    q, k, v = qkv.view(bsz, seqlen, 3, n_heads, d // n_heads).unbind(dim=2)
    return q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)


def _attn_masks(bsz: int, seqlen: int, device: torch.device, key_valid: torch.Tensor | None) -> torch.Tensor:
    """``[B or 1, 1, T, T]`` bool: True where a score is masked (future key, or padded key)."""
    masked = torch.ones(seqlen, seqlen, dtype=torch.bool, device=device).triu(1)[None, None]
    if key_valid is not None:
        masked = masked | ~key_valid.bool().view(bsz, 1, 1, seqlen)
    return masked


def attn_fwd(
    qkv: torch.Tensor,
    bsz: int,
    seqlen: int,
    n_heads: int,
    dropout_p: float = 0.0,
    dropout_seed: int = 0,
    key_valid: torch.Tensor | None = None,
) -> tuple[torch.Tensor, torch.Tensor]:
    """Causal attention over packed ``qkv`` ``[B*T, 3d]`` with optional probability dropout and
    key-padding mask ``key_valid`` ``[B, T]`` (reference ``models/gpt.py:56-69``).

    Returns ``out`` ``[B*T, d]`` (dtype of qkv) and ``lse`` ``[B, H, T]`` fp32 (undropped).  A
    query row with no unmasked key gets ``out = 0`` and ``lse = +inf`` (it is a padded position,
    whose branch output the caller zeroes anyway — reference ``gpt.py:73-74``).
    """
    q, k, v = (t.float() for t in _split_qkv(qkv, bsz, seqlen, n_heads))
    hd = q.shape[-1]
    s = (q @ k.transpose(-2, -1)) / math.sqrt(hd)
    s = s.masked_fill(_attn_masks(bsz, seqlen, qkv.device, key_valid), float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    lse = torch.where(torch.isfinite(lse), lse, torch.full_like(lse, float("inf")))
    p = torch.exp(s - lse[..., None])
    thr, dscale = dropout_params(dropout_p)
    if thr:
        keep = attn_dropout_keep(dropout_seed, dropout_p, bsz, n_heads, seqlen, qkv.device)
        p = torch.where(keep, p * dscale, torch.zeros_like(p))
    out = (p @ v).transpose(1, 2).reshape(bsz * seqlen, n_heads * hd)
    return out.to(qkv.dtype), lse


def attn_bwd(
    dout: torch.Tensor,
    qkv: torch.Tensor,
    out: torch.Tensor,
    lse: torch.Tensor,
    bsz: int,
    seqlen: int,
    n_heads: int,
    dropout_p: float = 0.0,
    dropout_seed: int = 0,
    key_valid: torch.Tensor | None = None,
) -> torch.Tensor:
    """Gradient of :func:`attn_fwd` w.r.t. packed ``qkv``; returns ``[B*T, 3d]`` in qkv dtype."""
    q, k, v = (t.float() for t in _split_qkv(qkv, bsz, seqlen, n_heads))
    hd = q.shape[-1]
    scale = 1.0 / math.sqrt(hd)
    do = dout.float().view(bsz, seqlen, n_heads, hd).transpose(1, 2)
    o = out.float().view(bsz, seqlen, n_heads, hd).transpose(1, 2)
    s = (q @ k.transpose(-2, -1)) * scale
    p = torch.exp(s - lse[..., None]).masked_fill(_attn_masks(bsz, seqlen, qkv.device, key_valid), 0.0)
    thr, dscale = dropout_params(dropout_p)
    keep = attn_dropout_keep(dropout_seed, dropout_p, bsz, n_heads, seqlen, qkv.device) if thr else None
    pd = p if keep is None else torch.where(keep, p * dscale, torch.zeros_like(p))
    dv = pd.transpose(-2, -1) @ do
    dp = do @ v.transpose(-2, -1)
    if keep is not None:
        dp = torch.where(keep, dp * dscale, torch.zeros_like(dp))
    delta = (do * o).sum(dim=-1, keepdim=True)
    ds = p * (dp - delta) * scale
    dq = ds @ k
    dk = ds.transpose(-2, -1) @ q
    dqkv = torch.stack([dq, dk, dv], dim=2)  # [B, H, 3, T, hd]
    dqkv = dqkv.permute(0, 3, 2, 1, 4).reshape(bsz * seqlen, 3 * n_heads * hd)
    return dqkv.to(qkv.dtype)


def sumsq(x: torch.Tensor) -> torch.Tensor:
    """Σ x² in fp32 as a 0-d tensor."""
    return x.float().pow(2).sum()


def clip_coef(sumsq_t: torch.Tensor, max_norm: float) -> torch.Tensor:
    """``[norm, coef]``: ``coef = min(1, max_norm / (norm + 1e-6))``, NaN for a non-finite norm."""
    norm = torch.sqrt(sumsq_t.float().reshape(1))
    coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
    coef = torch.where(torch.isfinite(norm), coef, torch.full_like(coef, float("nan")))
    return torch.cat([norm, coef])


def adamw_flat(
    param: torch.Tensor,
    grad: torch.Tensor,
    exp_avg: torch.Tensor,
    exp_avg_sq: torch.Tensor,
    shadow: torch.Tensor | None,
    *,
    lr: float,
    beta1: float,
    beta2: float,
    eps: float,
    weight_decay: float,
    step: int,
    grad_scale: torch.Tensor | None,
    skipped: torch.Tensor | None = None,
) -> None:
    """One decoupled-weight-decay Adam step over flat fp32 buffers (torch.optim.AdamW math).

    ``grad_scale`` (0-d fp32) multiplies the gradient first (gradient clipping without a host
    sync). When ``shadow`` is given, the updated parameters are also written to it (bf16 copy
    used by the compute path); ``shadow`` may be longer than ``param`` (padding is untouched).
    A non-finite ``grad_scale`` skips the step; ``skipped`` (int32 ``[total, consecutive]``)
    counts skips like the HIP kernel.
    """
    if grad_scale is not None and not bool(torch.isfinite(grad_scale).all()):
        if skipped is not None:
            skipped += 1
        return
    if skipped is not None:
        skipped[1] = 0
    g = grad if grad_scale is None else grad * grad_scale
    param.mul_(1.0 - lr * weight_decay)
    exp_avg.lerp_(g, 1.0 - beta1)
    exp_avg_sq.mul_(beta2).addcmul_(g, g, value=1.0 - beta2)
    bc1 = 1.0 - beta1**step
    bc2 = 1.0 - beta2**step
    denom = (exp_avg_sq.sqrt() / math.sqrt(bc2)).add_(eps)
    param.addcdiv_(exp_avg, denom, value=-lr / bc1)
    if shadow is not None:
        shadow[: param.numel()].copy_(param)
