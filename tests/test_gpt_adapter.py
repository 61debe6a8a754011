"""GPT adapter contract (reference tests/test_gpt_adapter.py)."""

from __future__ import annotations

import math

import pytest
import torch

from llmtrain.config.schemas import RunConfig
from llmtrain.data.tokenizer import ByteLevelTokenizer, get_gpt2_tokenizer
from llmtrain.models.base import LazyFloat
from llmtrain.models.gpt import GPT, GPTAdapter

from conftest import minimal_payload


def _cfg(**model) -> RunConfig:  # type: ignore[no-untyped-def]
    m = {"name": "gpt", "vocab_size": 64, "block_size": 16, "d_model": 64, "n_layers": 2, "n_heads": 2,
         "d_ff": 128, "dropout": 0.0}
    m.update(model)
    return RunConfig.model_validate(minimal_payload(model=m))


def _batch(b=2, t=16, v=64):  # type: ignore[no-untyped-def]
    ids = torch.randint(0, v, (b, t))
    return {"input_ids": ids, "labels": torch.roll(ids, -1, 1), "attention_mask": torch.ones_like(ids)}


def test_finite_loss_and_lazy_metric() -> None:
    adapter = GPTAdapter()
    model = adapter.build_model(_cfg())
    loss, metrics = adapter.compute_loss(model, _batch())
    assert loss.dim() == 0 and math.isfinite(loss.item())
    assert isinstance(metrics["loss"], LazyFloat)
    assert math.isfinite(metrics["loss"]) and abs(float(metrics["loss"]) - loss.item()) < 1e-6
    assert f"{metrics['loss']:.2f}"


def test_label_sensitivity_and_masking() -> None:
    adapter = GPTAdapter()
    torch.manual_seed(0)
    model = adapter.build_model(_cfg())
    batch = _batch()
    l1, _ = adapter.compute_loss(model, batch)
    other = dict(batch, labels=(batch["labels"] + 1) % 64)
    l2, _ = adapter.compute_loss(model, other)
    assert l1.item() != l2.item()
    masked = dict(batch, attention_mask=torch.zeros_like(batch["input_ids"]))
    with pytest.raises(ValueError, match="no valid target tokens"):
        adapter.compute_loss(model, masked)


@pytest.mark.parametrize(
    "batch,msg",
    [
        ({"input_ids": torch.zeros(4, dtype=torch.long), "labels": torch.zeros(4, dtype=torch.long)}, "2D"),
        ({"input_ids": torch.zeros(2, 4, dtype=torch.long), "labels": torch.zeros(2, 5, dtype=torch.long)}, "same shape"),
        ({"input_ids": torch.zeros(2, 4), "labels": torch.zeros(2, 4)}, "torch.long"),
        ({"input_ids": torch.zeros(2, 1, dtype=torch.long), "labels": torch.zeros(2, 1, dtype=torch.long)}, ">= 2"),
    ],
)
def test_batch_validation(batch, msg) -> None:  # type: ignore[no-untyped-def]
    adapter = GPTAdapter()
    with pytest.raises(ValueError, match=msg):
        adapter.compute_loss(adapter.build_model(_cfg()), batch)


def test_hyperparameters_honoured() -> None:
    model = GPTAdapter().build_model(_cfg(d_model=128, n_layers=3, n_heads=4, d_ff=256, block_size=32))
    assert isinstance(model, GPT)
    assert len(model.blocks) == 3 and model.blocks[0].attn.n_heads == 4
    assert model.blocks[0].mlp_fc.out_features == 256 and model.position_embedding.num_embeddings == 32


def test_vocab_from_tokenizer_and_roundtrip() -> None:
    tok = get_gpt2_tokenizer()
    assert tok.n_vocab == 50257
    model = GPTAdapter().build_model(_cfg(vocab_size=None))
    assert model.token_embedding.num_embeddings == tok.n_vocab
    text = "hello MI355X"
    assert tok.decode(tok.encode(text)) == text
    assert ByteLevelTokenizer().encode("a") == [97]
