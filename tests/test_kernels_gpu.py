"""Numerics of every gfx950 HIP kernel against the plain-PyTorch fp32 oracle of the same op
(``llmtrain.ops.reference``).  Inputs are random (never zero-filled) and shapes cover both the
GPT-2 124M production sizes and ragged/small edge cases."""

from __future__ import annotations

import math

import pytest
import torch

from llmtrain.ops import reference as ref

pytestmark = pytest.mark.gpu


def hip():
    return torch.ops.llmtrain_hip


def _close(a, b, atol, rtol, what=""):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol).sum().item()
    assert bad == 0, f"{what}: {bad} elements out of tolerance, max err {err.max().item():.3e}"


@pytest.mark.parametrize("M,d", [(4096, 768), (37, 64), (513, 1600)])
@pytest.mark.parametrize("with_delta", [False, True])
def test_add_layernorm_fwd(gpu_device, M, d, with_delta):
    g = torch.Generator(device="cpu").manual_seed(M + d)
    x = torch.randn(M, d, generator=g).to(gpu_device)
    delta = torch.randn(M, d, generator=g).to(gpu_device, torch.bfloat16) if with_delta else None
    w = (1 + 0.1 * torch.randn(d, generator=g)).to(gpu_device)
    b = (0.1 * torch.randn(d, generator=g)).to(gpu_device)
    xs, y, mu, rs = hip().add_layernorm_fwd(x, delta, w, b, 1e-5, torch.bfloat16)
    xs_r, y_r, mu_r, rs_r = ref.add_layernorm_fwd(x, delta, w, b, 1e-5, torch.float32)
    if with_delta:
        _close(xs, xs_r, 1e-6, 1e-6, "xs")
    _close(mu, mu_r, 1e-5, 1e-5, "mean")
    _close(rs, rs_r, 1e-4, 1e-4, "rstd")
    _close(y, y_r, 2e-2, 1e-2, "y(bf16)")


@pytest.mark.parametrize("M,d", [(4096, 768), (4099, 768), (100, 64), (777, 384), (513, 1600)])
@pytest.mark.parametrize("with_proj,lowp", [(True, True), (False, False), (False, True)])
def test_layernorm_bwd(gpu_device, M, d, with_proj, lowp):
    """Every LayerNorm-backward variant (the lean kernel for d <= 768, the general one above)
    against the fp32 reference: with / without the
    projection-bias column sum and the bf16 copy, odd row counts (dead rows of a 2-row wave)."""
    g = torch.Generator(device="cpu").manual_seed(7)
    x = torch.randn(M, d, generator=g).to(gpu_device)
    w = (1 + 0.1 * torch.randn(d, generator=g)).to(gpu_device)
    b = torch.zeros(d).to(gpu_device)
    _, _, mu, rs = ref.add_layernorm_fwd(x, None, w, b, 1e-5, torch.float32)
    dy = torch.randn(M, d, generator=g).to(gpu_device, torch.bfloat16)
    dres = torch.randn(M, d, generator=g).to(gpu_device)
    scale = torch.tensor(0.5, device=gpu_device)
    dw, db, dp = (torch.full((d,), 0.25, device=gpu_device) for _ in range(3))
    dw_r, db_r, dp_r = dw.clone(), db.clone(), dp.clone()
    dx, dx_lp = hip().layernorm_bwd(dy, x, mu, rs, w, dres, dw, db, scale, lowp, dp if with_proj else None)
    dx_r = ref.layernorm_bwd(dy, x, mu, rs, w, dres, dw_r, db_r, scale)
    ref.colsum_accum(dx_r, dp_r)
    _close(dx, dx_r, 1e-4, 1e-4, "dx")
    if lowp:
        _close(dx_lp, dx_r, 2e-2, 1e-2, "dx_lp")
    _close(dw, dw_r, 1e-2, 1e-4, "dgamma")
    _close(db, db_r, 1e-2, 1e-4, "dbeta")
    if with_proj:
        _close(dp, dp_r, 2e-2, 1e-4, "dproj")
    else:
        assert torch.equal(dp, torch.full((d,), 0.25, device=gpu_device))


@pytest.mark.parametrize("M,d", [(4096, 768), (4099, 768), (513, 1600), (100, 64)])
@pytest.mark.parametrize("mode", ["bf16_grad", "bf16"])
@pytest.mark.parametrize("drop", [0.0, 0.2])
def test_layernorm_bf16_residual_streams(gpu_device, M, d, mode, drop):
    """The engine's bf16 residual options (model.extra.residual_dtype): a bf16 residual stream in
    the forward (x, xs bf16; statistics of the rounded sum) and a bf16 gradient stream in the
    backward (dresid in, dx out), against the fp32 reference fed the same bf16 values; without
    dropout the bf16 GEMM operand IS dx (one buffer)."""
    g = torch.Generator(device="cpu").manual_seed(M + d)
    res_dt = torch.bfloat16 if mode == "bf16" else torch.float32
    x = torch.randn(M, d, generator=g).to(gpu_device, res_dt)
    delta = torch.randn(M, d, generator=g).to(gpu_device, torch.bfloat16)
    w = (1 + 0.1 * torch.randn(d, generator=g)).to(gpu_device)
    b = (0.1 * torch.randn(d, generator=g)).to(gpu_device)
    seed = ref.dropout_site_seed(5, 3)
    xs, y, mu, rs = hip().add_layernorm_fwd(x, delta, w, b, 1e-5, torch.bfloat16, drop, seed)
    xs_r, y_r, mu_r, rs_r = ref.add_layernorm_fwd(x, delta, w, b, 1e-5, torch.float32, drop, seed)
    assert xs.dtype == res_dt
    _close(xs, xs_r, 1e-6, 1e-6 if mode != "bf16" else 0.0, "xs")  # the same rounding
    _close(mu, mu_r, 1e-5, 1e-5, "mean")
    _close(rs, rs_r, 1e-4, 1e-4, "rstd")
    _close(y, y_r, 2e-2, 1e-2, "y")

    dy = torch.randn(M, d, generator=g).to(gpu_device, torch.bfloat16)
    dres = torch.randn(M, d, generator=g).to(gpu_device, torch.bfloat16)
    scale = torch.tensor(0.5, device=gpu_device)
    dw, db = torch.zeros(d, device=gpu_device), torch.zeros(d, device=gpu_device)
    dw_r, db_r = dw.clone(), db.clone()
    dx, dx_lp = hip().layernorm_bwd(dy, xs, mu, rs, w, dres, dw, db, scale, True, None, drop, seed, True)
    dx_r = ref.layernorm_bwd(dy, xs, mu, rs, w, dres, dw_r, db_r, scale, torch.float32)
    assert dx.dtype == torch.bfloat16
    _close(dx, dx_r, 1e-2, 8e-3, "dx (bf16 stream)")
    _close(dx_lp, ref._apply_dropout(dx.float(), drop, seed), 1e-2, 8e-3, "dx_lp")
    if drop == 0.0:
        assert dx_lp.data_ptr() == dx.data_ptr()  # the operand is the stream itself
    _close(dw, dw_r, 1e-2, 1e-4, "dgamma")
    _close(db, db_r, 1e-2, 1e-4, "dbeta")
    # embedding forward straight into a bf16 residual stream
    ids = torch.randint(0, 300, (2, 64), generator=g).to(gpu_device)
    wte = torch.randn(300, d, generator=g).to(gpu_device)
    wpe = torch.randn(64, d, generator=g).to(gpu_device)
    e = hip().embedding_fwd(ids, wte, wpe, drop, seed, True)
    assert e.dtype == torch.bfloat16
    assert torch.equal(e, ref.embedding_fwd(ids, wte, wpe, drop, seed, torch.bfloat16))


@pytest.mark.parametrize("M,V,Vp", [(256, 50257, 50304), (1000, 50257, 50304), (64, 16, 64), (33, 1000, 1024)])
def test_cross_entropy_fwd_bwd(gpu_device, M, V, Vp):
    g = torch.Generator(device="cpu").manual_seed(V)
    logits = (3 * torch.randn(M, Vp, generator=g)).to(gpu_device, torch.bfloat16)
    labels = torch.randint(0, V, (M,), generator=g).to(gpu_device)
    labels[3] = -100  # ignored row
    w = torch.rand(M, generator=g).to(gpu_device) / M
    lg_r = logits.float().clone()
    loss_r = ref.cross_entropy_fwd_bwd(lg_r, labels, V, w)
    lg = logits.clone()
    loss = hip().cross_entropy_fwd_bwd(lg, labels, V, w)
    _close(loss, loss_r, 1e-3, 1e-4, "loss")
    _close(lg, lg_r, 1e-6, 2e-2, "dlogits")
    assert torch.all(lg[:, V:] == 0)


@pytest.mark.parametrize("M,F", [(2048, 3072), (40000, 3072), (1001, 200)])
def test_gelu_fwd_bwd(gpu_device, M, F):
    g = torch.Generator(device="cpu").manual_seed(3)
    u = (2 * torch.randn(M, F, generator=g)).to(gpu_device, torch.bfloat16)
    _close(hip().gelu_fwd(u), ref.gelu_fwd(u.float()), 1e-2, 1e-2, "gelu")
    dg = torch.randn(M, F, generator=g).to(gpu_device, torch.bfloat16)
    dbias = torch.zeros(F, device=gpu_device)
    dbias_r = torch.zeros(F, device=gpu_device)
    du = hip().gelu_bwd(dg, u, dbias)
    du_r = ref.gelu_bwd(dg.float(), u.float(), dbias_r)
    _close(du, du_r, 2e-2, 2e-2, "du")
    _close(dbias, dbias_r, 0.3 * (M / 2048) ** 0.5, 1e-2, "dbias")  # rounding noise grows ~sqrt(M)
    # and exactly (up to fp32 summation order) the column sums of the bf16 du the kernel wrote
    _close(dbias, du.float().sum(0), 1e-2, 1e-4, "dbias vs colsum(du)")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_colsum(gpu_device, dtype):
    g = torch.Generator(device="cpu").manual_seed(4)
    dy = torch.randn(1000, 2304, generator=g).to(gpu_device, dtype)
    out = torch.ones(2304, device=gpu_device)
    out_r = out.clone()
    hip().colsum_accum(dy, out)
    ref.colsum_accum(dy, out_r)
    _close(out, out_r, 1e-2, 1e-4, "colsum")


def test_embedding(gpu_device):
    g = torch.Generator(device="cpu").manual_seed(5)
    B, T, d, V = 4, 128, 768, 5000
    ids = torch.randint(0, V, (B, T), generator=g).to(gpu_device)
    ids[0, :10] = 7  # repeated token: atomics must accumulate
    wte = torch.randn(V, d, generator=g).to(gpu_device)
    wpe = torch.randn(256, d, generator=g).to(gpu_device)
    _close(hip().embedding_fwd(ids, wte, wpe), ref.embedding_fwd(ids, wte, wpe), 1e-6, 1e-6, "emb fwd")
    dx = torch.randn(B * T, d, generator=g).to(gpu_device)
    dwte, dwpe = torch.zeros_like(wte), torch.zeros_like(wpe)
    dwte_r, dwpe_r = dwte.clone(), dwpe.clone()
    hip().embedding_bwd(dx, ids, dwte, dwpe)
    ref.embedding_bwd(dx, ids, dwte_r, dwpe_r)
    _close(dwte, dwte_r, 1e-4, 1e-5, "dwte")
    _close(dwpe, dwpe_r, 1e-4, 1e-5, "dwpe")


@pytest.mark.parametrize("det", [False, True])
def test_embedding_bwd_bf16_stream(gpu_device, det):
    """The embedding backward reads a bf16 residual-stream gradient as is (atomic scatter and the
    deterministic sorted scatter): equal to the fp32 oracle on the same bf16 values."""
    g = torch.Generator(device="cpu").manual_seed(15)
    B, T, d, V = 4, 128, 768, 3000
    ids = torch.randint(0, V, (B, T), generator=g).to(gpu_device)
    ids[1, :20] = 11
    dx = torch.randn(B * T, d, generator=g).to(gpu_device, torch.bfloat16)
    dwte, dwpe = torch.zeros(V, d, device=gpu_device), torch.zeros(256, d, device=gpu_device)
    dwte_r, dwpe_r = dwte.clone(), dwpe.clone()
    prev = hip().get_deterministic()
    hip().set_deterministic(det)
    try:
        hip().embedding_bwd(dx, ids, dwte, dwpe)
    finally:
        hip().set_deterministic(prev)
    ref.embedding_bwd(dx.float(), ids, dwte_r, dwpe_r)
    _close(dwte, dwte_r, 1e-4, 1e-5, "dwte bf16 dx")
    _close(dwpe, dwpe_r, 1e-4, 1e-5, "dwpe bf16 dx")


def test_sumsq_and_adamw(gpu_device):
    g = torch.Generator(device="cpu").manual_seed(6)
    n = 1_000_003  # ragged tail
    p = torch.randn(n, generator=g).to(gpu_device)
    grad = torch.randn(n, generator=g).to(gpu_device)
    m = (0.1 * torch.randn(n, generator=g)).to(gpu_device)
    v = torch.rand(n, generator=g).to(gpu_device) * 0.01
    s = hip().sumsq(grad)
    assert math.isclose(float(s), float(grad.double().pow(2).sum()), rel_tol=1e-5)
    scale = torch.tensor(0.7, device=gpu_device)
    shadow = torch.zeros(n + 64, device=gpu_device, dtype=torch.bfloat16)
    p_r, m_r, v_r = p.clone(), m.clone(), v.clone()
    kw = dict(lr=3e-4, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.1, step=7)
    hip().adamw_flat(p, grad, m, v, shadow, kw["lr"], kw["beta1"], kw["beta2"], kw["eps"], kw["weight_decay"], kw["step"], scale)
    ref.adamw_flat(p_r, grad, m_r, v_r, None, grad_scale=scale, **kw)
    _close(p, p_r, 1e-6, 1e-5, "param")
    _close(m, m_r, 1e-7, 1e-5, "exp_avg")
    _close(v, v_r, 1e-9, 1e-4, "exp_avg_sq")  # fma vs mul+add: 1 ulp-level
    _close(shadow[:n], p_r, 1e-2, 1e-2, "shadow")
    assert torch.all(shadow[n:] == 0)


@pytest.mark.parametrize("offset", [1, 2, 3])
@pytest.mark.parametrize("n", [1, 2, 3, 5, 1_000_003])
def test_sumsq_unaligned_views(gpu_device, offset, n):
    """Bucket views of the flat gradient may start off a 16-byte boundary: the scalar head."""
    g = torch.Generator(device="cpu").manual_seed(offset * 7 + n)
    base = torch.randn(n + 8, generator=g).to(gpu_device)
    x = base[offset : offset + n]
    assert math.isclose(float(hip().sumsq(x)), float(x.double().pow(2).sum()), rel_tol=1e-5, abs_tol=1e-12)


@pytest.mark.parametrize("n", [4096, 1_000_003])  # tiled kernel / grid-stride kernel (ragged)
def test_adamw_skips_nonfinite_step(gpu_device, n):
    """A NaN/Inf global norm: clip_coef returns a NaN coefficient and the AdamW kernel writes
    nothing (weights, moments, shadow unchanged) and counts the skip on device; a finite step then
    resets the consecutive counter."""
    g = torch.Generator(device="cpu").manual_seed(9)
    p = torch.randn(n, generator=g).to(gpu_device)
    grad = torch.randn(n, generator=g).to(gpu_device)
    m = (0.1 * torch.randn(n, generator=g)).to(gpu_device)
    v = torch.rand(n, generator=g).to(gpu_device) * 0.01
    shadow = p.to(torch.bfloat16)
    before = [t.clone() for t in (p, m, v, shadow)]
    skipped = torch.zeros(2, dtype=torch.int32, device=gpu_device)
    args = (1e-2, 0.9, 0.999, 1e-8, 0.1, 3)
    for bad in (float("nan"), float("inf")):
        out = hip().clip_coef(torch.tensor([bad], device=gpu_device), 1.0)
        assert math.isnan(float(out[1]))
        hip().adamw_flat(p, grad, m, v, shadow, *args, out[1], None, skipped)
    assert all(torch.equal(a, b) for a, b in zip((p, m, v, shadow), before))
    assert skipped.tolist() == [2, 2]
    out = hip().clip_coef(torch.tensor([16.0], device=gpu_device), 1.0)
    assert torch.equal(out.cpu(), ref.clip_coef(torch.tensor(16.0), 1.0))
    hip().adamw_flat(p, grad, m, v, shadow, *args, out[1], None, skipped)
    p_r, m_r, v_r = before[0].clone(), before[1].clone(), before[2].clone()
    ref.adamw_flat(p_r, grad, m_r, v_r, None, lr=1e-2, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.1, step=3,
                   grad_scale=out[1])
    _close(p, p_r, 1e-6, 1e-5, "param after the applied step")
    assert skipped.tolist() == [2, 0]


def test_adamw_matches_torch_adamw(gpu_device):
    """Several steps of the fused kernel track torch.optim.AdamW (the reference optimizer)."""
    g = torch.Generator(device="cpu").manual_seed(8)
    p0 = torch.randn(4096, generator=g)
    p = p0.clone().to(gpu_device)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    tp = torch.nn.Parameter(p0.clone().to(gpu_device))
    opt = torch.optim.AdamW([tp], lr=1e-2, weight_decay=0.1)
    for step in range(1, 6):
        grad = torch.randn(4096, generator=g).to(gpu_device)
        tp.grad = grad.clone()
        opt.step()
        hip().adamw_flat(p, grad, m, v, None, 1e-2, 0.9, 0.999, 1e-8, 0.1, step, None)
    _close(p, tp.detach(), 1e-6, 1e-5, "adamw vs torch")


@pytest.mark.parametrize("B,T,H", [(2, 1024, 12), (1, 256, 2), (2, 200, 3), (1, 70, 1)])
def test_attention_fwd_bwd(gpu_device, B, T, H):
    g = torch.Generator(device="cpu").manual_seed(B * T + H)
    d = 64 * H
    qkv = torch.randn(B * T, 3 * d, generator=g).to(gpu_device, torch.bfloat16)
    out, lse = hip().attn_fwd(qkv, B, T, H)
    out_r, lse_r = ref.attn_fwd(qkv.float(), B, T, H)
    _close(lse, lse_r, 2e-3, 1e-3, "lse")
    _close(out, out_r, 2e-2, 2e-2, "out")
    dout = torch.randn(B * T, d, generator=g).to(gpu_device, torch.bfloat16)
    dqkv = hip().attn_bwd(dout, qkv, out, lse, B, T, H)
    dqkv_r = ref.attn_bwd(dout.float(), qkv.float(), out.float(), lse, B, T, H)
    names = ["dq", "dk", "dv"]
    a = dqkv.float().view(B, T, 3, H, 64)
    r = dqkv_r.view(B, T, 3, H, 64)
    for i, name in enumerate(names):
        scale = r[:, :, i].abs().max().item()
        _close(a[:, :, i], r[:, :, i], 2e-2 * scale, 3e-2, name)
    # fused qkv-bias gradient (column sums of dqkv) accumulates into an existing buffer
    dbias = torch.ones(3 * d, device=gpu_device)
    dqkv2 = hip().attn_bwd(dout, qkv, out, lse, B, T, H, 0.0, 0, dbias)
    assert torch.equal(dqkv2, dqkv)
    want = 1.0 + dqkv_r.sum(dim=0)
    _close(dbias, want, 2e-2 * want.abs().max().item(), 2e-2, "qkv bias grad")


def test_attention_causality(gpu_device):
    """Changing future tokens never changes earlier outputs (reference tests/test_gpt_model.py:11-40)."""
    g = torch.Generator(device="cpu").manual_seed(11)
    B, T, H = 1, 256, 2
    qkv = torch.randn(B * T, 3 * 64 * H, generator=g).to(gpu_device, torch.bfloat16)
    out1, _ = hip().attn_fwd(qkv, B, T, H)
    qkv2 = qkv.clone()
    qkv2[200:] = torch.randn(56, 3 * 64 * H, generator=g).to(gpu_device, torch.bfloat16)
    out2, _ = hip().attn_fwd(qkv2, B, T, H)
    assert torch.equal(out1[:200], out2[:200])


@pytest.mark.parametrize("M,d", [(4096, 768), (513, 1600)])
def test_layernorm_bwd_deferred_params_batched(gpu_device, M, d):
    """A block's two LayerNorm backwards with their dgamma / dbeta partial rows reduced by ONE
    ln_param_reduce launch give exactly (bitwise) what the immediate per-LayerNorm reduce gives."""
    g = torch.Generator(device="cpu").manual_seed(3)
    outs = {}
    for mode in ("immediate", "deferred"):
        dst, parts = [], []
        for k in range(2):
            gk = torch.Generator(device="cpu").manual_seed(100 + k)
            x = torch.randn(M, d, generator=gk).to(gpu_device)
            w = (1 + 0.1 * torch.randn(d, generator=gk)).to(gpu_device)
            _, _, mu, rs = ref.add_layernorm_fwd(x, None, w, torch.zeros(d, device=gpu_device), 1e-5, torch.float32)
            dy = torch.randn(M, d, generator=gk).to(gpu_device, torch.bfloat16)
            dw, db = torch.full((d,), 0.5, device=gpu_device), torch.full((d,), -0.5, device=gpu_device)
            if mode == "immediate":
                dx, _ = hip().layernorm_bwd(dy, x, mu, rs, w, None, dw, db, None, True, None)
            else:
                dx, _, pr = hip().layernorm_bwd_deferred(dy, x, mu, rs, w, None, dw, db, None, True)
                parts.append(pr)
                assert torch.equal(dw, torch.full((d,), 0.5, device=gpu_device))  # not yet reduced
            dst += [dw, db]
            dst.append(dx)
        if parts:
            hip().ln_param_reduce(parts, [dst[0], dst[1], dst[3], dst[4]])
        outs[mode] = dst
    for a, b in zip(outs["immediate"], outs["deferred"]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("mode", [-1, 0, 2])
@pytest.mark.parametrize("M,N,K,lda", [(4096, 768, 768, 768), (2048, 2304, 768, 2304), (1000, 200, 72, 200),
                                        (3000, 1000, 768, 1024), (2080, 1600, 4800, 1600),
                                        (1500, 1001, 768, 1024), (101, 768, 768, 768),
                                        (2048, 50257, 768, 50304),  # the LM head's padded logits
                                        # K tails of 64 / 128 columns -> 512 x 64 strip tiles
                                        (2048, 1600, 1600, 1600), (3000, 6400, 1600, 6400), (101, 1600, 1600, 1600),
                                        (1200, 512, 640, 512),
                                        # N tail, whole K -> swapped operands, transposed output
                                        (2500, 1600, 6400, 1600), (1500, 320, 2304, 320),
                                        (1500, 320, 2304, 384)])  # lda > N: bias call unswapped, split=3 call swapped
def test_wgrad_gemm_pp(gpu_device, M, N, K, lda, mode):
    """Ping-pong weight-gradient GEMM (csrc/gemm_wgrad_pp.hip): dst += dY^T X and bias += colsum(dY)
    against fp32, for the auto plan, the slab (deterministic) and the atomic epilogue, ragged M/N/K,
    a column-slice dY (row stride lda > N), a single-stage chunk and an odd stage count (the
    zero-padded last stage), the K-tail strip tiles and the swapped (transposed-output) plan."""
    g = torch.Generator(device="cpu").manual_seed(M + N + K + mode)
    dy = torch.randn(M, lda, generator=g).to(gpu_device, torch.bfloat16)[:, :N]
    x = torch.randn(M, K, generator=g).to(gpu_device, torch.bfloat16)
    c = torch.randn(N, K, generator=g).to(gpu_device)
    b = torch.randn(N, generator=g).to(gpu_device)
    want = c + dy.float().t() @ x.float()
    want_b = b + dy.float().sum(0)
    hip().wgrad_gemm_pp(dy, x, c, b, 0, mode)
    _close(c, want, 2e-5 * want.abs().max().item(), 1e-4, "wgrad_pp")
    _close(b, want_b, 2e-5 * want_b.abs().max().item(), 1e-4, "wgrad_pp bias")
    # an explicit split and no bias
    c2 = torch.zeros(N, K, device=gpu_device)
    hip().wgrad_gemm_pp(dy, x, c2, None, 3, mode)
    _close(c2, dy.float().t() @ x.float(), 2e-5 * want.abs().max().item(), 1e-4, "wgrad_pp split=3")


@pytest.mark.parametrize("N,K", [(2304, 768), (6400, 1600), (1600, 6400)])
def test_wgrad_gemm_pp_slabs_bitwise(gpu_device, N, K):
    """The slab epilogue reduces the split partials in a fixed order: repeated launches are equal
    bit for bit (the deterministic mode needs no separate path) — also with strip tiles (6400 x
    1600) and the swapped plan with its separate bias pass (1600 x 6400)."""
    g = torch.Generator(device="cpu").manual_seed(5)
    dy = torch.randn(16384, N, generator=g).to(gpu_device, torch.bfloat16)
    x = torch.randn(16384, K, generator=g).to(gpu_device, torch.bfloat16)
    outs = []
    for _ in range(3):
        c = torch.zeros(N, K, device=gpu_device)
        b = torch.zeros(N, device=gpu_device)
        hip().wgrad_gemm_pp(dy, x, c, b, 0, 0)
        outs.append((c, b))
    for c, b in outs[1:]:
        assert torch.equal(c, outs[0][0]) and torch.equal(b, outs[0][1])


@pytest.mark.parametrize("M,N,K", [(4096, 1600, 1600), (4096, 4800, 1600), (4096, 1600, 6400)])
def test_wgrad_gemm_pp_tail_tiling_vs_square_tiles(gpu_device, M, N, K):
    """The d = 1600 tilings (strips / swapped operands) against the 256 x 256-only plan (mode + 8)
    and fp32: both within the same bound of the fp32 product, bias included."""
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    dy = torch.randn(M, N, generator=g).to(gpu_device, torch.bfloat16)
    x = torch.randn(M, K, generator=g).to(gpu_device, torch.bfloat16)
    want = dy.float().t() @ x.float()
    want_b = dy.float().sum(0)
    for mode in (0, 8):
        c = torch.zeros(N, K, device=gpu_device)
        b = torch.zeros(N, device=gpu_device)
        hip().wgrad_gemm_pp(dy, x, c, b, 0, mode)
        _close(c, want, 2e-5 * want.abs().max().item(), 1e-4, f"wgrad_pp mode {mode}")
        _close(b, want_b, 2e-5 * want_b.abs().max().item(), 1e-4, f"wgrad_pp bias mode {mode}")


# ---- fused forward / dX GEMM (csrc/gemm_fused.hip) -------------------------------------------
GEMM_SHAPES = [(4096, 3072, 768), (8192, 3072, 768), (513, 768, 3072), (1000, 200, 256), (300, 2304, 768),
               (65536 + 96, 768, 256)]  # >= kWideM m-tiles: one raster band over all of N, ragged M


def _gemm_operands(M, N, K, b_kn, dev, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    a = (torch.randn(M, K, generator=g) / math.sqrt(K)).to(dev, torch.bfloat16)
    w = torch.randn(N, K, generator=g).to(dev, torch.bfloat16)  # nn.Linear weight [out, in]
    b = w.t().contiguous() if b_kn else w  # b_kn: the [K, N] operand of dX = dY @ W
    bias = (0.1 * torch.randn(N, generator=g)).to(dev, torch.bfloat16)
    return a, w, b, bias


@pytest.mark.parametrize("M,N,K", GEMM_SHAPES)
@pytest.mark.parametrize("b_kn", [False, True])
def test_gemm_fused_bias(gpu_device, M, N, K, b_kn):
    a, w, b, bias = _gemm_operands(M, N, K, b_kn, gpu_device, M + N + K)
    out, none = hip().gemm_fused(a, b, b_kn, 0, bias)
    assert none is None
    ref_out = a.float() @ w.float().t() + bias.float()
    _close(out, ref_out, 2e-2, 1e-2, "gemm+bias")
    out_nb, _ = hip().gemm_fused(a, b, b_kn, 0)
    _close(out_nb, a.float() @ w.float().t(), 2e-2, 1e-2, "gemm")
    again, _ = hip().gemm_fused(a, b, b_kn, 0, bias)
    assert torch.equal(out, again), "gemm_fused is not deterministic (pipeline race?)"
    # out=: written in place into a row slice of a larger tensor, rows around it untouched
    big = torch.full((M + 16, N), 7.0, device=gpu_device, dtype=torch.bfloat16)
    ret, _ = hip().gemm_fused(a, b, b_kn, 0, bias, None, None, 0, big[8 : 8 + M])
    assert ret.data_ptr() == big[8].data_ptr()
    assert torch.equal(big[8 : 8 + M], out)
    assert torch.all(big[:8] == 7.0) and torch.all(big[8 + M :] == 7.0)


@pytest.mark.parametrize("M,N,K", GEMM_SHAPES)
@pytest.mark.parametrize("b_kn", [False, True])
def test_gemm_fused_bias_gelu(gpu_device, M, N, K, b_kn):
    a, w, b, bias = _gemm_operands(M, N, K, b_kn, gpu_device, 3 * M + K)
    u, gl = hip().gemm_fused(a, b, b_kn, 1, bias)
    u_ref = a.float() @ w.float().t() + bias.float()
    _close(u, u_ref, 2e-2, 1e-2, "u")
    # GELU is applied to the bf16 pre-activation the backward will see
    _close(gl, torch.nn.functional.gelu(u.float()), 1e-2, 1e-2, "gelu(u)")


@pytest.mark.parametrize("M,N,K", GEMM_SHAPES)
@pytest.mark.parametrize("b_kn", [True, False])
def test_gemm_fused_dgelu(gpu_device, M, N, K, b_kn):
    a, w, b, _ = _gemm_operands(M, N, K, b_kn, gpu_device, 5 * M + N)
    g = torch.Generator(device="cpu").manual_seed(11)
    u = (2 * torch.randn(M, N, generator=g)).to(gpu_device, torch.bfloat16)
    dbias = torch.full((N,), 0.5, device=gpu_device)
    du, none = hip().gemm_fused(a, b, b_kn, 2, None, u, dbias)
    assert none is None
    uf = u.float().requires_grad_(True)
    gelu_grad = torch.autograd.grad(torch.nn.functional.gelu(uf).sum(), uf)[0]
    du_ref = (a.float() @ w.float().t()) * gelu_grad
    _close(du, du_ref, 2e-2, 1e-2, "du")
    # the bias gradient sums exactly the bf16 values written
    _close(dbias, 0.5 + du.float().sum(0), 1e-3, 1e-4, "dbias")


@pytest.mark.parametrize("M,N,K", GEMM_SHAPES)
@pytest.mark.parametrize("b_kn", [False, True])
def test_gemm_fused_gelu_and_derivative(gpu_device, M, N, K, b_kn):
    """Epilogue 4: gelu'(u) and gelu(u) of the bf16 u = a @ w^T + bias (one erf evaluation);
    epilogue 5: (dy @ W) * stored gelu'(u) with the bias column sums — together equal to
    epilogue 1 + epilogue 2 up to the bf16 rounding of the stored derivative."""
    a, w, b, bias = _gemm_operands(M, N, K, b_kn, gpu_device, 9 * M + K)
    gd, gl = hip().gemm_fused(a, b, b_kn, 4, bias)
    u, gl1 = hip().gemm_fused(a, b, b_kn, 1, bias)
    assert torch.equal(gl, gl1)  # the same GELU of the same bf16 u
    _close(gd, ref.gelu_grad(u.float()), 1e-2, 1e-2, "gelu'(u)")
    dy, wd, bd, _ = _gemm_operands(M, N, K, not b_kn, gpu_device, 11 * M + N)
    db5, db2 = torch.zeros(N, device=gpu_device), torch.zeros(N, device=gpu_device)
    du5, none = hip().gemm_fused(dy, bd, not b_kn, 5, None, gd, db5)
    assert none is None
    du2, _ = hip().gemm_fused(dy, bd, not b_kn, 2, None, u, db2)
    du_ref = (dy.float() @ wd.float().t()) * ref.gelu_grad(u.float()).float()
    _close(du5, du_ref, 2e-2, 2e-2, "du (stored gelu')")
    _close(du5, du2, 2e-2, 2e-2, "du: epilogue 5 vs 2")
    _close(db5, du5.float().sum(0), 1e-3, 1e-4, "dbias sums the written values")


@pytest.mark.parametrize(
    "M,N,K,T",
    [(4096, 768, 768, 1024), (1536, 768, 768, 512), (600, 256, 256, 300), (2048, 1600, 1600, 256),
     (131072, 768, 768, 1024)],  # the benchmark's shape: wide raster band + non-temporal stores
)
@pytest.mark.parametrize("b_kn", [True, False])
def test_gemm_fused_attn_dx_delta(gpu_device, M, N, K, T, b_kn):
    """Epilogue 3: dO = dY @ W plus the attention backward's delta = per-head rowsum(dO * O) and
    the V-bias colsum(dO); delta must equal what the attention backward's own pass computes."""
    a, w, b, _ = _gemm_operands(M, N, K, b_kn, gpu_device, 7 * M + N)
    g = torch.Generator(device="cpu").manual_seed(13)
    o = torch.randn(M, N, generator=g).to(gpu_device, torch.bfloat16)
    dbias = torch.full((N,), 0.25, device=gpu_device)
    do, delta = hip().gemm_fused(a, b, b_kn, 3, None, o, dbias, T)
    _close(do, a.float() @ w.float().t(), 2e-2, 1e-2, "dO")
    H = N // 64
    ref_delta = (do.float() * o.float()).view(M // T, T, H, 64).sum(-1).permute(0, 2, 1)
    assert delta.shape == (M // T, H, T)
    _close(delta, ref_delta, 1e-3, 1e-3, "delta")
    ref_b = 0.25 + do.float().sum(0)
    _close(dbias, ref_b, 1e-3 + 1e-5 * ref_b.abs().max().item(), 1e-4, "dbias_v")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_scale_device_scalar(gpu_device, dtype):
    """``scale``: x * s with s read from device memory, fp32 math and one rounding — matches the
    fp32 product rounded once (the LM-head weight-gradient operand ``go * hf``)."""
    g = torch.Generator(device="cpu").manual_seed(7)
    x = torch.randn(1001, 768, generator=g).to(gpu_device, dtype)
    s = torch.tensor(1.0 / 3.0, device=gpu_device)
    y = hip().scale(x, s.reshape(1))
    want = (x.float() * s).to(dtype)
    assert y.dtype == dtype and y.shape == x.shape
    assert torch.equal(y, want)
