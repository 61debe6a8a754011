"""Flash-attention kernels (csrc/attention_{fwd,bwd}.hip) against an INDEPENDENT oracle: fp32
autograd of eager attention (reference ``models/gpt.py:56-74``: scores / sqrt(hd), causal and
key-padding masks, softmax, P V) on the same bf16 inputs — no kernel output (lse, O) is fed into
the oracle.  Covers head dims 32 / 48 / 64 (the reference presets and GPT-2) and 128, GPT-2 XL's 25 heads,
a production-sized batch (B*T = 64K tokens), ragged T, and key-padding masks with left padding
(query rows that see no valid key), right padding and holes."""

from __future__ import annotations

import math

import pytest
import torch

from llmtrain import ops

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("gpu_device")]


def hip():
    return torch.ops.llmtrain_hip


def _oracle(qkv: torch.Tensor, B: int, T: int, H: int, key_valid: torch.Tensor | None, dout: torch.Tensor):
    """fp32 autograd: returns (out [B*T, H*hd], dqkv [B*T, 3*H*hd], live [B, T] rows with a valid key)."""
    hd = qkv.shape[1] // (3 * H)
    x = qkv.float().detach().requires_grad_(True)
    q, k, v = (t.transpose(1, 2) for t in x.view(B, T, 3, H, hd).unbind(dim=2))
    s = (q @ k.transpose(-2, -1)) / math.sqrt(hd)
    masked = torch.ones(T, T, dtype=torch.bool, device=qkv.device).triu(1)[None, None]
    if key_valid is not None:
        masked = masked | ~key_valid.bool()[:, None, None, :]
    s = s.masked_fill(masked, torch.finfo(torch.float32).min)  # reference's mask value
    out = (torch.softmax(s, dim=-1) @ v).transpose(1, 2).reshape(B * T, H * hd)
    live = (~masked).any(dim=-1)[:, 0].expand(B, T)  # [B, T]
    out.backward(dout.float())
    return out.detach(), x.grad.detach(), live


def _check(name: str, got: torch.Tensor, want: torch.Tensor, rows_dim_last: int, slack: float = 6e-2) -> None:
    got, want = got.float(), want.float()
    # tensor-wide: relative Frobenius error (bf16 operands, fp32 accumulation)
    rel = (got - want).norm() / want.norm().clamp_min(1e-12)
    assert rel < 1.5e-2, f"{name}: relative error {rel:.3e}"
    # per row (each token's vector): catches a single wrong row that a tensor-wide norm would hide
    g2, w2 = got.reshape(-1, rows_dim_last), want.reshape(-1, rows_dim_last)
    row_err = (g2 - w2).norm(dim=1)
    row_ref = w2.norm(dim=1)
    bad = row_err > 3e-2 * row_ref + slack * row_ref.mean()  # rows that cancel to ~0 (dq of query 0)
    assert not bool(bad.any()), f"{name}: {int(bad.sum())} rows off, first {bad.nonzero()[:4].flatten().tolist()}"


CASES = [
    # B, T, H, hd, padding
    (2, 1024, 12, 64, None),
    (1, 1024, 25, 64, None),  # GPT-2 XL heads
    (64, 1024, 12, 64, None),  # B*T = 64K tokens (production micro-batch scale)
    (2, 256, 8, 32, None),  # K8s ConfigMap / gpt_smoke head dim
    (2, 256, 8, 48, None),  # gpt_wikitext_better head dim
    (3, 200, 2, 32, None),  # ragged T
    (1, 70, 1, 64, None),
    (2, 8, 4, 16, None),  # gpt_smoke's block size: one partial 64-key tile
    (3, 33, 2, 64, "mixed"),
    (1, 2, 2, 64, None),  # (T = 1 makes dQ identically zero: no relative error to check)
    (3, 300, 4, 64, "mixed"),
    (3, 256, 8, 48, "mixed"),
    (4, 128, 8, 32, "mixed"),  # the K8s ConfigMap model's attention with padding
    (2, 1024, 12, 64, "mixed"),
    (2, 1024, 8, 128, None),  # head dim 128: two 64-wide halves, the 4-wave backward
    (1, 70, 2, 128, None),
    (3, 300, 4, 128, "mixed"),
    # B*H filling the CUs evenly: the per-(b, h) workgroup with fp32 dQ accumulation (the smaller
    # grids above take the per-key-block split with bf16 partial planes + reduce)
    (32, 300, 8, 48, "mixed"),
    (20, 1024, 12, 64, "mixed"),
    # B*H = 512 = two per CU on 256 CUs: the 4-wave / two-workgroups-per-CU backward where built
    # (csrc/attention_bwd.hip kBwdFourWaves), else the per-(b, h) 8-wave form
    (64, 256, 8, 64, None),
    (32, 300, 16, 64, "mixed"),
    (64, 160, 8, 32, "mixed"),
]


def _mask(B: int, T: int, kind: str | None, device) -> torch.Tensor | None:
    if kind is None:
        return None
    m = torch.ones(B, T, dtype=torch.long)
    m[0, T - T // 3 :] = 0  # right padding
    if B > 1:
        m[1, : T // 4 + 3] = 0  # left padding: those queries see no valid key
    if B > 2:
        m[2, 5] = 0
        m[2, T // 2 : T // 2 + 70] = 0  # holes, one spanning a 64-key tile boundary
    return m.to(device)


@pytest.mark.parametrize("B,T,H,hd,pad", CASES)
def test_attention_matches_autograd(gpu_device, B: int, T: int, H: int, hd: int, pad: str | None) -> None:
    g = torch.Generator(device="cpu").manual_seed(B * T + H + hd)
    d = H * hd
    qkv = torch.randn(B * T, 3 * d, generator=g).to(gpu_device, torch.bfloat16)
    mask = _mask(B, T, pad, gpu_device)
    km = None if mask is None else ops.attn_key_masks(mask)
    dout = torch.randn(B * T, d, generator=g).to(gpu_device, torch.bfloat16)
    if mask is not None:  # the engine zeroes the attention branch of padded queries: no gradient there
        dout = dout * mask.reshape(-1, 1).to(dout.dtype)

    out, lse = hip().attn_fwd(qkv, B, T, H, 0.0, 0, None if km is None else km[0])
    dbias = torch.zeros(3 * d, device=gpu_device)
    dqkv = hip().attn_bwd(dout, qkv, out, lse, B, T, H, 0.0, 0, dbias, None, None if km is None else km[1])
    out_r, dqkv_r, live = _oracle(qkv, B, T, H, mask, dout)

    live_rows = live.reshape(-1)
    _check("out", out[live_rows], out_r[live_rows], hd)
    if not bool(live_rows.all()):  # rows without a valid key: O = 0, lse = +inf
        assert torch.all(out[~live_rows] == 0)
        assert torch.all(torch.isinf(lse.permute(0, 2, 1).reshape(-1, H)[~live_rows]))
    a = dqkv.float().view(B * T, 3, H, hd)
    r = dqkv_r.view(B * T, 3, H, hd)
    for i, name in enumerate(("dq", "dk", "dv")):
        _check(name, a[:, i], r[:, i], hd)
    assert torch.isfinite(dqkv.float()).all()
    # fused qkv-bias gradient == column sums of the dqkv the kernel wrote
    torch.testing.assert_close(dbias, dqkv.float().sum(0), atol=2e-2 * dbias.abs().max().item() + 1e-3, rtol=1e-2)


def test_last_key_gradients(gpu_device) -> None:
    """dK/dV of the last key (T - 1) of a sequence: regression test for a K/V load descriptor that
    ended inside row T - 1 and read that key's K and V as zeros."""
    B, T, H, hd = 1, 128, 2, 64
    g = torch.Generator(device="cpu").manual_seed(5)
    qkv = torch.randn(B * T, 3 * H * hd, generator=g).to(gpu_device, torch.bfloat16)
    dout = torch.zeros(B * T, H * hd, device=gpu_device, dtype=torch.bfloat16)
    dout[T - 1] = torch.randn(H * hd, generator=g).to(gpu_device, torch.bfloat16)  # only the last query
    out, lse = hip().attn_fwd(qkv, B, T, H)
    dqkv = hip().attn_bwd(dout, qkv, out, lse, B, T, H)
    _, dqkv_r, _ = _oracle(qkv, B, T, H, None, dout)
    a, r = dqkv.float().view(T, 3, H, hd), dqkv_r.view(T, 3, H, hd)
    for i in (1, 2):  # dK, dV of key T-1
        torch.testing.assert_close(a[T - 1, i], r[T - 1, i], atol=2e-2 * r[T - 1, i].abs().max().item(), rtol=3e-2)


def test_padding_does_not_change_valid_rows(gpu_device) -> None:
    """Right padding: the valid prefix's outputs equal the unpadded run over that prefix."""
    B, T, H, hd, L = 2, 320, 4, 64, 200
    g = torch.Generator(device="cpu").manual_seed(9)
    qkv = torch.randn(B * T, 3 * H * hd, generator=g).to(gpu_device, torch.bfloat16)
    mask = torch.ones(B, T, dtype=torch.long, device=gpu_device)
    mask[:, L:] = 0
    km = ops.attn_key_masks(mask)
    out, _ = hip().attn_fwd(qkv, B, T, H, 0.0, 0, km[0])
    prefix = qkv.view(B, T, -1)[:, :L].reshape(B * L, -1).contiguous()
    out_p, _ = hip().attn_fwd(prefix, B, L, H)
    torch.testing.assert_close(out.view(B, T, -1)[:, :L].float(), out_p.view(B, L, -1).float(), atol=0, rtol=0)


@pytest.mark.parametrize("hd,B,T,H", [(64, 2, 200, 3), (128, 2, 200, 3), (64, 64, 300, 4)])
def test_attention_dropout_head_dims(gpu_device, hd: int, B: int, T: int, H: int) -> None:
    """Probability dropout at head dims 64 and 128 (and, B*H = 256, the per-(b, h) backward grid)
    against fp32 AUTOGRAD of eager dropout attention (reference ``models/gpt.py:56-69`` with
    ``attn_dropout`` on the probabilities).  Only the keep mask is shared with the kernel — the
    counter hash of ``ops/reference.attn_dropout_keep``, which any correct implementation must
    reproduce bit for bit; the oracle forms its own softmax, lse, O and gradients from the bf16
    inputs, so no kernel output (O, lse) feeds it."""
    from llmtrain.ops import reference as ref

    g = torch.Generator(device="cpu").manual_seed(hd)
    qkv = torch.randn(B * T, 3 * hd * H, generator=g).to(torch.bfloat16)
    dout = torch.randn(B * T, hd * H, generator=g).to(torch.bfloat16)
    p_drop, seed = 0.25, ref.dropout_site_seed(11, 8)
    out_g, lse_g = ops.attn_fwd(qkv.to(gpu_device), B, T, H, dropout=(p_drop, seed))
    dbias = torch.zeros(3 * hd * H, device=gpu_device)
    dq_g = ops.attn_bwd(dout.to(gpu_device), qkv.to(gpu_device), out_g, lse_g, B, T, H, dropout=(p_drop, seed),
                        qkv_bias_grad=dbias).cpu().float()

    # independent oracle: fp32 eager attention with the mask applied to the probabilities
    keep = ref.attn_dropout_keep(seed, p_drop, B, H, T, torch.device("cpu"))  # [B, H, T, T]
    x = qkv.float().detach().requires_grad_(True)
    q, k, v = (t.transpose(1, 2) for t in x.view(B, T, 3, H, hd).unbind(dim=2))
    s = (q @ k.transpose(-2, -1)) / math.sqrt(hd)
    causal = torch.ones(T, T, dtype=torch.bool).triu(1)[None, None]
    s = s.masked_fill(causal, torch.finfo(torch.float32).min)
    lse_r = torch.logsumexp(s, dim=-1)  # the undropped normaliser the kernel stores
    _, dscale = ref.dropout_params(p_drop)  # 1 / keep probability of the 16-bit threshold
    probs = torch.where(keep, torch.softmax(s, dim=-1) * dscale, torch.zeros(()))
    out_r = (probs @ v).transpose(1, 2).reshape(B * T, H * hd)
    out_r.backward(dout.float())
    dq_r = x.grad

    torch.testing.assert_close(lse_g.cpu(), lse_r, atol=2e-3, rtol=2e-3)
    _check("out (dropout)", out_g.cpu(), out_r.detach(), hd)
    a, r = dq_g.view(B * T, 3, H, hd), dq_r.view(B * T, 3, H, hd)
    # dq of query 0 is exactly 0 in exact arithmetic (one key: dS = P (dP - delta) = 0); the kernel's
    # delta comes from the bf16 O, whose rounding the 1 / keep-probability scale amplifies
    for i, name in enumerate(("dq", "dk", "dv")):
        _check(f"{name} (dropout)", a[:, i], r[:, i], hd, slack=0.15)
    want = dq_r.sum(dim=0)
    assert (dbias.cpu() - want).abs().max().item() < 2e-2 * want.abs().max().item()
