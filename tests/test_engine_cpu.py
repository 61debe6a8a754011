"""The fused engine's hand-written backward, flat parameter store and fused AdamW, verified on
CPU against PyTorch autograd + torch.optim.AdamW (the reference's training math)."""

from __future__ import annotations

import copy

import pytest
import torch
import torch.nn.functional as F

from llmtrain.models.gpt import GPT
from llmtrain.training.optim import FusedAdamW, fused_clip_coef


def _pair(**kw):  # type: ignore[no-untyped-def]
    torch.manual_seed(0)
    args = dict(vocab_size=100, block_size=16, d_model=64, n_layers=2, n_heads=4, d_ff=128, dropout=0.0)
    args.update(kw)
    ref = GPT(**args)
    fused = copy.deepcopy(ref)
    fused.prepare_runtime(compute_dtype=torch.float32)
    return ref, fused


@pytest.mark.parametrize("tie", [True, False])
def test_fused_backward_matches_autograd(tie: bool) -> None:
    ref, fused = _pair(tie_embeddings=tie)
    ids = torch.randint(0, 100, (3, 16))
    labels = torch.randint(0, 100, (3, 16))
    loss_ref = F.cross_entropy(ref(ids).reshape(-1, 100), labels.reshape(-1))
    (loss_ref * 0.25).backward()
    fused.flat_store.zero_grad()
    loss = fused.fused_loss(ids, labels)
    (loss * 0.25).backward()
    assert abs(loss.item() - loss_ref.item()) < 1e-5
    for (name, p), (_, q) in zip(fused.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(p.grad, q.grad, atol=1e-6, rtol=1e-4, msg=name)


def test_fused_masked_loss_matches_masked_mean() -> None:
    ref, fused = _pair()
    ids = torch.randint(0, 100, (2, 16))
    mask = torch.ones(2, 16, dtype=torch.long)
    loss_ref = F.cross_entropy(ref(ids).reshape(-1, 100), ids.reshape(-1))
    with torch.no_grad():
        loss = fused.fused_loss(ids, ids, mask)
    assert abs(loss.item() - loss_ref.item()) < 1e-5


@pytest.mark.parametrize("n_heads", [4, 2])  # head dims 16 and 32
def test_fused_key_padding_matches_module_path(n_heads: int) -> None:
    """Key-padding mask (reference gpt.py:60-64 key masking + :73-74 zeroing of padded query rows)
    on the fused engine: loss and every gradient equal the module path's autograd, with left and
    right padding (rows whose keys are all padded included)."""
    ref, fused = _pair(n_heads=n_heads)
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(0, 100, (3, 16), generator=g)
    labels = torch.randint(0, 100, (3, 16), generator=g)
    mask = torch.ones(3, 16, dtype=torch.long)
    mask[0, 11:] = 0  # right padding
    mask[1, :5] = 0   # left padding: queries 0..4 see no valid key
    mask[2, 7] = 0    # a hole
    logits = ref(ids, attention_mask=mask)
    keep = mask.reshape(-1).bool()
    loss_ref = F.cross_entropy(logits.reshape(-1, 100), labels.reshape(-1), reduction="none")[keep].mean()
    loss_ref.backward()
    fused.flat_store.zero_grad()
    loss = fused.fused_loss(ids, labels, mask)
    loss.backward()
    assert abs(loss.item() - loss_ref.item()) < 1e-5
    for (name, p), (_, q) in zip(fused.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(p.grad, q.grad, atol=1e-6, rtol=1e-4, msg=name)


def test_gradient_accumulation_and_views() -> None:
    ref, fused = _pair()
    store = fused.flat_store
    for p in fused.parameters():
        assert p.grad is not None and p.grad.data_ptr() >= store.grad.data_ptr()
    ids = torch.randint(0, 100, (2, 16))
    for _ in range(2):
        (fused.fused_loss(ids, ids) / 2).backward()
        (F.cross_entropy(ref(ids).reshape(-1, 100), ids.reshape(-1)) / 2).backward()
    for p, q in zip(fused.parameters(), ref.parameters()):
        torch.testing.assert_close(p.grad, q.grad, atol=1e-6, rtol=1e-4)


def test_fused_adamw_matches_torch_and_state_layout() -> None:
    ref, fused = _pair()
    opt_ref = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.1)
    opt = FusedAdamW(fused.parameters(), store=fused.flat_store, lr=1e-2, weight_decay=0.1)
    ids = torch.randint(0, 100, (2, 16))
    for _ in range(3):
        opt_ref.zero_grad()
        opt.zero_grad()
        F.cross_entropy(ref(ids).reshape(-1, 100), ids.reshape(-1)).backward()
        torch.nn.utils.clip_grad_norm_(ref.parameters(), 0.5)
        opt_ref.step()
        fused.fused_loss(ids, ids).backward()
        norm, coef = fused_clip_coef(fused.flat_store, 0.5)
        opt.step(grad_scale=coef)
    # Adam normalises the update, so ~1e-7 gradient differences on near-zero-gradient entries
    # become ~1e-5 parameter differences after a few lr=1e-2 steps: compare at that scale.
    for p, q in zip(fused.parameters(), ref.parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), atol=1e-4, rtol=1e-4)
    sd, sd_ref = opt.state_dict(), opt_ref.state_dict()
    assert sd["param_groups"][0].keys() == sd_ref["param_groups"][0].keys()
    assert sd["state"].keys() == sd_ref["state"].keys()
    for i in sd["state"]:
        assert sd["state"][i].keys() == sd_ref["state"][i].keys()
        assert float(sd["state"][i]["step"]) == 3.0 and sd["state"][i]["step"].dtype == torch.float32
        torch.testing.assert_close(sd["state"][i]["exp_avg"], sd_ref["state"][i]["exp_avg"], atol=1e-6, rtol=1e-4)


def test_fused_adamw_loads_reference_optimizer_state() -> None:
    ref, fused = _pair()
    opt_ref = torch.optim.AdamW(ref.parameters(), lr=1e-3, weight_decay=0.0)
    ids = torch.randint(0, 100, (2, 16))
    F.cross_entropy(ref(ids).reshape(-1, 100), ids.reshape(-1)).backward()
    opt_ref.step()
    opt = FusedAdamW(fused.parameters(), store=fused.flat_store, lr=1e-3, weight_decay=0.0)
    opt.load_state_dict(opt_ref.state_dict())
    fused.load_state_dict(ref.state_dict())
    assert opt._step_count_host == 1
    p0 = next(fused.parameters())
    torch.testing.assert_close(opt.state[p0]["exp_avg"], opt_ref.state[next(ref.parameters())]["exp_avg"])
    assert opt.state[p0]["exp_avg"].data_ptr() >= opt.exp_avg.data_ptr()  # still a flat view


def test_shadow_tracks_master_version() -> None:
    _, fused = _pair()
    store = fused.flat_store
    assert not store.shadow_is_stale()
    with torch.no_grad():
        fused.ln_f.weight.fill_(2.0)
    assert store.shadow_is_stale()
    store.sync_shadow()
    assert torch.all(store.shadow_of(fused.ln_f.weight) == 2.0)
    head = store.shadow_of(fused.lm_head.weight, padded=True)
    assert head.shape[0] % 64 == 0 and torch.all(head[100:] == 0)


def test_state_dict_roundtrip_after_flattening() -> None:
    ref, fused = _pair()
    sd = fused.state_dict()
    assert set(sd) == set(ref.state_dict())
    fresh = GPT(vocab_size=100, block_size=16, d_model=64, n_layers=2, n_heads=4, d_ff=128, dropout=0.0)
    fresh.load_state_dict(sd)
    for p, q in zip(fresh.parameters(), ref.parameters()):
        torch.testing.assert_close(p, q)


@pytest.mark.parametrize("residual", ["bf16_grad", "bf16"])
def test_bf16_residual_streams_track_autograd(residual: str) -> None:
    """model.extra.residual_dtype on the engine's reference ops (bf16 compute): the residual stream
    and / or its gradient stored in bf16 stays within bf16 rounding of fp32 autograd, and the
    option is refused with an fp32 compute dtype."""
    torch.manual_seed(0)
    args = dict(vocab_size=100, block_size=16, d_model=64, n_layers=2, n_heads=4, d_ff=128, dropout=0.0)
    ref = GPT(**args)
    fused = copy.deepcopy(ref)
    engine = fused.prepare_runtime(compute_dtype=torch.bfloat16, residual=residual)
    assert engine.grad_dtype == torch.bfloat16
    assert engine.res_dtype == (torch.bfloat16 if residual == "bf16" else torch.float32)
    ids = torch.randint(0, 100, (3, 16))
    labels = torch.randint(0, 100, (3, 16))
    F.cross_entropy(ref(ids).reshape(-1, 100), labels.reshape(-1)).backward()
    fused.flat_store.zero_grad()
    fused.fused_loss(ids, labels).backward()
    for (name, p), (_, q) in zip(fused.named_parameters(), ref.named_parameters()):
        rel = ((p.grad.float() - q.grad).norm() / (q.grad.norm() + 1e-12)).item()
        assert rel < 3e-2, f"{name}: {rel:.3e}"
    with pytest.raises(ValueError, match="bf16 compute"):
        GPT(**args).prepare_runtime(compute_dtype=torch.float32, residual=residual)
    with pytest.raises(ValueError, match="residual_dtype"):
        GPT(**args).prepare_runtime(compute_dtype=torch.bfloat16, residual="fp16")


def test_mlp_store_gd_matches_u() -> None:
    """model.extra.mlp_store "gd": the fc forward keeps gelu'(u) and the projection dX multiplies
    by it — the same gradients as keeping u (fp32 reference ops: exactly the same math)."""
    ref, fused_u = _pair()
    fused_gd = copy.deepcopy(ref)
    fused_gd.prepare_runtime(compute_dtype=torch.float32, mlp_store="gd")
    ids = torch.randint(0, 100, (3, 16))
    labels = torch.randint(0, 100, (3, 16))
    for m in (fused_u, fused_gd):
        m.flat_store.zero_grad()
        m.fused_loss(ids, labels).backward()
    for (name, p), (_, q) in zip(fused_gd.named_parameters(), fused_u.named_parameters()):
        torch.testing.assert_close(p.grad, q.grad, atol=1e-6, rtol=1e-5, msg=name)
    with pytest.raises(ValueError, match="mlp_store"):
        GPT(vocab_size=10, block_size=4, d_model=8, n_layers=1, n_heads=2, d_ff=16, dropout=0.0).prepare_runtime(
            compute_dtype=torch.float32, mlp_store="x")
