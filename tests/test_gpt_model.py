"""GPT module numerics (reference tests/test_gpt_model.py) plus parameter-count / init /
state_dict layout pinned to the reference architecture."""

from __future__ import annotations

import pytest
import torch

from llmtrain.models.gpt import GPT


def _gpt(**kw) -> GPT:  # type: ignore[no-untyped-def]
    torch.manual_seed(0)
    args = dict(vocab_size=256, block_size=16, d_model=64, n_layers=2, n_heads=4, d_ff=256, dropout=0.0)
    args.update(kw)
    return GPT(**args).eval()


def test_attention_and_logits_causality() -> None:
    model = _gpt()
    x = torch.randint(0, 256, (2, 16))
    y = x.clone()
    y[:, 10:] = torch.randint(0, 256, (2, 6))
    with torch.no_grad():
        a, b = model(x), model(y)
        ha = model.blocks[0].attn(model.token_embedding(x))
        hb = model.blocks[0].attn(model.token_embedding(y))
    torch.testing.assert_close(a[:, :10], b[:, :10], atol=1e-6, rtol=0)
    torch.testing.assert_close(ha[:, :10], hb[:, :10], atol=1e-6, rtol=0)


def test_grads_reach_every_parameter() -> None:
    model = _gpt().train()
    model(torch.randint(0, 256, (2, 16))).sum().backward()
    for name, p in model.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all(), name
        assert p.grad.abs().sum() > 0, name


def test_shapes_tying_and_block_limit() -> None:
    model = _gpt()
    assert model(torch.randint(0, 256, (3, 7))).shape == (3, 7, 256)
    assert model.lm_head.weight is model.token_embedding.weight
    with pytest.raises(ValueError, match="exceeds block size"):
        model(torch.randint(0, 256, (1, 17)))


@pytest.mark.parametrize(
    "kw,count",
    [
        (dict(vocab_size=16, block_size=8, d_model=64, n_layers=2, n_heads=2, d_ff=128), 68_608),
        (dict(vocab_size=256, block_size=32, d_model=64, n_layers=2, n_heads=4, d_ff=256), 118_528 - 0),
        (dict(vocab_size=50257, block_size=1024, d_model=768, n_layers=12, n_heads=12, d_ff=3072), 124_439_808),
    ],
)
def test_parameter_counts_match_reference(kw, count) -> None:  # type: ignore[no-untyped-def]
    model = GPT(dropout=0.0, **kw)
    n = sum(p.numel() for p in model.parameters())
    if kw["vocab_size"] == 256:
        # notebook gpt_model_smoke: V=256 d=64 L=2 H=4 F=256 -> 118,528 with block 32
        assert n == count
    else:
        assert n == count


def test_state_dict_layout_and_init() -> None:
    model = GPT(vocab_size=128, block_size=16, d_model=64, n_layers=3, n_heads=4, d_ff=128, dropout=0.1)
    sd = model.state_dict()
    assert "blocks.0.attn.causal_mask" in sd and sd["blocks.0.attn.causal_mask"].dtype == torch.bool
    assert sd["blocks.0.attn.causal_mask"].shape == (1, 1, 16, 16)
    assert sd["lm_head.weight"].data_ptr() == sd["token_embedding.weight"].data_ptr()
    assert torch.all(sd["blocks.1.mlp_fc.bias"] == 0) and torch.all(sd["ln_f.weight"] == 1)
    std = model.blocks[0].attn.out_proj.weight.std().item()
    assert abs(std - 0.02 / (2 * 3) ** 0.5) < 0.004
    keys = {k for k in sd if k.startswith("blocks.0.")}
    assert keys == {
        "blocks.0.ln_1.weight", "blocks.0.ln_1.bias", "blocks.0.attn.qkv_proj.weight", "blocks.0.attn.qkv_proj.bias",
        "blocks.0.attn.out_proj.weight", "blocks.0.attn.out_proj.bias", "blocks.0.attn.causal_mask",
        "blocks.0.ln_2.weight", "blocks.0.ln_2.bias", "blocks.0.mlp_fc.weight", "blocks.0.mlp_fc.bias",
        "blocks.0.mlp_proj.weight", "blocks.0.mlp_proj.bias",
    }


def test_padding_mask_zeroes_padded_queries() -> None:
    model = _gpt()
    x = torch.randint(0, 256, (1, 16))
    mask = torch.ones(1, 16, dtype=torch.long)
    mask[0, 12:] = 0
    with torch.no_grad():
        out = model.blocks[0].attn(model.token_embedding(x), attention_mask=mask)
    assert torch.all(out[0, 12:] == 0)
