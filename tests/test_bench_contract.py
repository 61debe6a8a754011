"""bench.py driver contract on CPU: the config it builds for N ranks gives every rank whole
micro-batches of the configured size (a short DistributedSampler shard would silently shrink the
per-GPU batch at 8 GPUs), and it names the BASELINE.json metric."""

from __future__ import annotations

import argparse
import importlib.util
import json
from pathlib import Path

import pytest

from llmtrain.data.synthetic_tokens import SyntheticTokensDataModule

ROOT = Path(__file__).resolve().parents[1]


def _bench():
    spec = importlib.util.spec_from_file_location("bench_main", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    assert spec.loader is not None
    spec.loader.exec_module(mod)
    return mod


def test_metric_matches_baseline_json() -> None:
    assert _bench().BASELINE_METRIC == json.loads((ROOT / "BASELINE.json").read_text())["metric"]


@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("mb,accum", [(128, 1), (16, 2)])
def test_every_rank_gets_full_micro_batches(world: int, mb: int, accum: int) -> None:
    bench = _bench()
    args = argparse.Namespace(model="gpt2-124m", micro_batch=mb, grad_accum=accum, dropout=0.0,
                              path="fused", warmup=1, steps=2, bucket_mb=64.0)
    cfg = bench.make_config(args, world)
    n = cfg.data.extra["train_sequences"]
    assert n // world >= mb * accum
    # the last rank's shard through the real data module (world hinted via the ddp section);
    # a small vocab keeps the Markov table cheap, the sharding arithmetic is the same
    small = cfg.model_copy(update={
        "ddp": cfg.ddp.model_copy(update={"world_size": world, "rank": world - 1}),
        "model": cfg.model.model_copy(update={"vocab_size": 512, "block_size": 8}),
    })
    dm = SyntheticTokensDataModule()
    dm.setup(small, tokenizer=None)
    batch = next(iter(dm.train_dataloader()))
    assert batch["input_ids"].shape == (mb, 8)
