"""Data modules: dummy_text semantics (reference tests/test_dummy_text_data.py), synthetic_tokens
(MI355X benchmark data), hf_text with a fake ``datasets`` backend (reference
tests/test_hf_text_data.py: window shapes, label shift, processed cache, sampler hints)."""

from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest
import torch
from torch.utils.data.distributed import DistributedSampler

from llmtrain.config.schemas import RunConfig
from llmtrain.data.dummy_text import DummyTextDataModule
from llmtrain.data.hf_text import HFTextDataModule
from llmtrain.data.synthetic_tokens import SyntheticTokensDataModule, markov_streams

from conftest import minimal_payload


def _cfg(**over) -> RunConfig:  # type: ignore[no-untyped-def]
    return RunConfig.model_validate(minimal_payload(**over))


def test_dummy_text_shapes_and_copy_task() -> None:
    cfg = _cfg(model={"name": "dummy_gpt", "block_size": 32, "vocab_size": 50},
               trainer={"max_steps": 10, "micro_batch_size": 2, "warmup_steps": 0})
    dm = DummyTextDataModule()
    dm.setup(cfg)
    val = next(iter(dm.val_dataloader()))
    assert val["input_ids"].shape == (2, 8)
    assert torch.equal(val["input_ids"], val["labels"])
    assert len(dm._train) == 20 and len(dm._val) == 4
    a = next(iter(dm.train_dataloader()))
    b = next(iter(dm.train_dataloader()))
    assert torch.equal(a["input_ids"], b["input_ids"])  # deterministic
    with pytest.raises(RuntimeError):
        DummyTextDataModule().train_dataloader()


def test_dummy_text_sampler_from_config_hint() -> None:
    cfg = _cfg(ddp={"world_size": 2, "rank": 1})
    dm = DummyTextDataModule()
    dm.setup(cfg)
    assert isinstance(dm.train_dataloader().sampler, DistributedSampler)


def test_markov_streams_are_learnable() -> None:
    s = markov_streams(8, 50, 100, branching=2, seed=1, table_seed=2)
    assert s.shape == (8, 50) and s.max() < 100
    # each token has at most `branching` successors
    succ: dict[int, set[int]] = {}
    for row in s:
        for a, b in zip(row[:-1], row[1:]):
            succ.setdefault(int(a), set()).add(int(b))
    assert max(len(v) for v in succ.values()) <= 2
    np.testing.assert_array_equal(s, markov_streams(8, 50, 100, branching=2, seed=1, table_seed=2))


def test_synthetic_tokens_windows() -> None:
    cfg = _cfg(model={"name": "gpt", "block_size": 64, "vocab_size": 300},
               data={"name": "synthetic_tokens", "extra": {"train_sequences": 16, "val_sequences": 4}},
               trainer={"micro_batch_size": 4, "max_steps": 5, "warmup_steps": 0})
    dm = SyntheticTokensDataModule()
    dm.setup(cfg)
    batch = next(iter(dm.train_dataloader()))
    assert batch["input_ids"].shape == (4, 64) and batch["input_ids"].dtype == torch.long
    assert torch.equal(batch["input_ids"][:, 1:], batch["labels"][:, :-1])  # next-token shift
    assert torch.all(batch["attention_mask"] == 1)
    assert len(dm.val_dataloader().dataset) == 4


def test_synthetic_tokens_needs_vocab() -> None:
    cfg = _cfg(model={"name": "gpt"}, data={"name": "synthetic_tokens"})
    with pytest.raises(ValueError, match="vocab_size"):
        SyntheticTokensDataModule().setup(cfg)


class _ToyTokenizer:
    def encode(self, text: str) -> list[int]:
        return [ord(c) % 50 for c in text]


@pytest.fixture
def fake_datasets(monkeypatch: pytest.MonkeyPatch):
    datasets = pytest.importorskip("datasets")
    calls = {"n": 0}

    def fake_load_dataset(name, config, split, cache_dir):  # type: ignore[no-untyped-def]
        calls["n"] += 1
        texts = ["abcdefghij" * 3, None, "klmnopqrstuvwxyz" * 2, ""]
        return datasets.Dataset.from_dict({"text": texts})

    monkeypatch.setattr(datasets, "load_dataset", fake_load_dataset)
    return calls


def test_hf_text_windows_cache_and_loaders(tmp_path: Path, fake_datasets) -> None:  # type: ignore[no-untyped-def]
    cfg = _cfg(
        model={"name": "gpt", "block_size": 8, "vocab_size": 64},
        data={"name": "hf_text", "dataset_name": "fake/ds", "dataset_config": "cfg", "text_column": "text",
              "cache_dir": str(tmp_path), "num_workers": 0},
        trainer={"micro_batch_size": 2, "max_steps": 5, "warmup_steps": 0},
    )
    dm = HFTextDataModule()
    dm.setup(cfg, tokenizer=_ToyTokenizer())
    row = dm._train_dataset[0]
    assert len(row["input_ids"]) == 8 and row["input_ids"][1:] == row["labels"][:-1]
    cache = tmp_path / "processed" / "fake__ds__cfg__b8__train"
    assert cache.exists()
    before = fake_datasets["n"]
    HFTextDataModule().setup(cfg, tokenizer=_ToyTokenizer())
    assert fake_datasets["n"] == before  # served from the processed cache
    batch = next(iter(dm.train_dataloader()))
    assert batch["input_ids"].shape == (2, 8) and batch["attention_mask"].dtype == torch.long


def test_hf_text_setup_errors() -> None:
    dm = HFTextDataModule()
    with pytest.raises(ValueError, match="dataset_name"):
        dm.setup(_cfg(data={"name": "hf_text"}), tokenizer=_ToyTokenizer())
    with pytest.raises(ValueError, match="text_column"):
        dm.setup(_cfg(data={"name": "hf_text", "dataset_name": "x"}), tokenizer=_ToyTokenizer())
    with pytest.raises(ValueError, match="tokenizer"):
        dm.setup(_cfg(data={"name": "hf_text", "dataset_name": "x", "text_column": "t"}), tokenizer=None)
