"""Fused dropout (reference gpt.py: embedding ``drop``, ``attn_dropout``, ``resid_dropout``,
``mlp_dropout``): the engine's counter-based masks against an autograd re-implementation of the
model that applies the SAME masks (llmtrain.ops.reference), keep-rate statistics, determinism,
and eval mode switching it off.  GPU tests check each HIP kernel's mask and math against the
reference ops bit-for-bit on the mask."""

from __future__ import annotations

import copy

import pytest
import torch
import torch.nn.functional as F

from llmtrain.models.gpt import GPT
from llmtrain.ops import reference as ref


def _functional_loss(model: GPT, ids: torch.Tensor, labels: torch.Tensor, p: float, step_seed: int) -> torch.Tensor:
    def site(k: int) -> tuple[float, int]:
        return (p, ref.dropout_site_seed(step_seed, k))

    B, T = ids.shape
    H = model.n_heads
    x = ref.embedding_fwd(ids, model.token_embedding.weight, model.position_embedding.weight, *site(0))
    for i, blk in enumerate(model.blocks):
        h = F.layer_norm(x, (model.d_model,), blk.ln_1.weight, blk.ln_1.bias, blk.ln_1.eps)
        att, _ = ref.attn_fwd(F.linear(h, blk.attn.qkv_proj.weight, blk.attn.qkv_proj.bias), B, T, H, *site(2 + 3 * i))
        x = x + ref._apply_dropout(F.linear(att, blk.attn.out_proj.weight, blk.attn.out_proj.bias), *site(1 + 3 * i))
        h2 = F.layer_norm(x, (model.d_model,), blk.ln_2.weight, blk.ln_2.bias, blk.ln_2.eps)
        g = F.gelu(F.linear(h2, blk.mlp_fc.weight, blk.mlp_fc.bias))
        x = x + ref._apply_dropout(F.linear(g, blk.mlp_proj.weight, blk.mlp_proj.bias), *site(3 + 3 * i))
    hf = F.layer_norm(x, (model.d_model,), model.ln_f.weight, model.ln_f.bias, model.ln_f.eps)
    logits = hf @ model.lm_head.weight.t()
    return F.cross_entropy(logits, labels.reshape(-1))


def _pair(p: float):  # type: ignore[no-untyped-def]
    torch.manual_seed(0)
    ref_model = GPT(vocab_size=96, block_size=16, d_model=64, n_layers=2, n_heads=4, d_ff=128, dropout=p)
    fused = copy.deepcopy(ref_model)
    fused.prepare_runtime(compute_dtype=torch.float32)
    return ref_model, fused


@pytest.mark.parametrize("p", [0.1, 0.35])
def test_fused_dropout_matches_autograd_with_same_masks(p: float) -> None:
    ref_model, fused = _pair(p)
    ids = torch.randint(0, 96, (3, 16))
    labels = torch.randint(0, 96, (3, 16))
    torch.manual_seed(1234)
    step_seed = int(torch.randint(0, 2**31 - 1, (1,)).item())
    want = _functional_loss(ref_model, ids, labels, p, step_seed)
    want.backward()
    fused.train()
    fused.flat_store.zero_grad()
    torch.manual_seed(1234)  # the engine draws the same step seed
    got = fused.fused_loss(ids, labels)
    got.backward()
    assert abs(got.item() - want.item()) < 1e-5
    no_drop = _functional_loss(ref_model, ids, labels, 0.0, 0).item()
    assert abs(got.item() - no_drop) > 1e-4  # the masks really changed the loss
    for (name, a), (_, b) in zip(fused.named_parameters(), ref_model.named_parameters()):
        torch.testing.assert_close(a.grad, b.grad, atol=2e-6, rtol=1e-4, msg=name)


def test_eval_mode_disables_fused_dropout() -> None:
    ref_model, fused = _pair(0.3)
    ids = torch.randint(0, 96, (2, 16))
    fused.eval()
    with torch.no_grad():
        a = fused.fused_loss(ids, ids).item()
        b = fused.fused_loss(ids, ids).item()
    assert a == b
    assert abs(a - _functional_loss(ref_model, ids, ids, 0.0, 0).item()) < 1e-5


def test_mask_statistics_and_site_independence() -> None:
    thr, scale = ref.dropout_params(0.1)
    idx = torch.arange(1 << 18)
    k1 = ref.dropout_keep(ref.dropout_site_seed(5, 1), thr, idx)
    k2 = ref.dropout_keep(ref.dropout_site_seed(5, 2), thr, idx)
    assert abs(k1.float().mean().item() - 0.9) < 0.005
    assert abs((k1 & k2).float().mean().item() - 0.81) < 0.006  # independent sites
    assert abs(scale - 1.0 / (1.0 - thr / 65536)) < 1e-9
    keep = ref.attn_dropout_keep(77, 0.2, 2, 3, 32, "cpu")
    assert keep.shape == (2, 3, 32, 32) and abs(keep.float().mean().item() - 0.8) < 0.03
    assert not torch.equal(keep[0, 0], keep[0, 1])  # per-(b, h) planes differ


# ---- GPU: each kernel's mask and math against the reference ops ----------------------------------


@pytest.mark.gpu
def test_dropout_mask_kernel_matches_reference(gpu_device) -> None:  # type: ignore[no-untyped-def]
    seed = ref.dropout_site_seed(99, 4)
    thr, _ = ref.dropout_params(0.15)
    got = torch.ops.llmtrain_hip.dropout_mask(1 << 20, 0.15, seed, torch.empty(1, device=gpu_device)).cpu()
    assert torch.equal(got, ref.dropout_keep(seed, thr, torch.arange(1 << 20)))


@pytest.mark.gpu
def test_fused_dropout_kernels_on_gpu(gpu_device) -> None:  # type: ignore[no-untyped-def]
    from llmtrain import ops

    g = torch.Generator().manual_seed(3)
    M, d = 512, 256
    x = torch.randn(M, d, generator=g)
    delta = torch.randn(M, d, generator=g)
    w, b = torch.randn(d, generator=g), torch.randn(d, generator=g)
    drop = (0.2, ref.dropout_site_seed(11, 7))
    xs_g, y_g, _, _ = ops.add_layernorm_fwd(x.to(gpu_device), delta.to(gpu_device), w.to(gpu_device),
                                             b.to(gpu_device), 1e-5, torch.float32, dropout=drop)
    xs_r, y_r, _, _ = ref.add_layernorm_fwd(x, delta, w, b, 1e-5, torch.float32, *drop)
    torch.testing.assert_close(xs_g.cpu(), xs_r, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(y_g.cpu(), y_r, atol=1e-4, rtol=1e-4)
    # attention with probability dropout: forward and backward
    B, T, H = 2, 200, 3
    qkv = torch.randn(B * T, 3 * 64 * H, generator=g).to(torch.bfloat16)
    dout = torch.randn(B * T, 64 * H, generator=g).to(torch.bfloat16)
    adrop = (0.25, ref.dropout_site_seed(11, 8))
    out_g, lse_g = ops.attn_fwd(qkv.to(gpu_device), B, T, H, dropout=adrop)
    out_r, lse_r = ref.attn_fwd(qkv, B, T, H, *adrop)
    torch.testing.assert_close(lse_g.cpu(), lse_r, atol=2e-3, rtol=2e-3)
    torch.testing.assert_close(out_g.cpu().float(), out_r.float(), atol=3e-2, rtol=3e-2)
    dbias = torch.zeros(3 * 64 * H, device=gpu_device)
    dq_g = ops.attn_bwd(dout.to(gpu_device), qkv.to(gpu_device), out_g, lse_g, B, T, H, dropout=adrop,
                        qkv_bias_grad=dbias).cpu().float()
    dq_r = ref.attn_bwd(dout, qkv, out_g.cpu(), lse_g.cpu(), B, T, H, *adrop).float()
    scale = dq_r.abs().max().item()
    assert (dq_g - dq_r).abs().max().item() < 2e-2 * scale
    want = dq_r.sum(dim=0)  # K part: exactly 0 in exact arithmetic (softmax shift invariance)
    assert (dbias.cpu() - want).abs().max().item() < 2e-2 * want.abs().max().item()
