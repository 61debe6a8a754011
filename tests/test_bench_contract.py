"""bench.py driver contract on CPU: the config it builds for N ranks gives every rank whole
micro-batches of the configured size (a short DistributedSampler shard would silently shrink the
per-GPU batch at 8 GPUs), and it names the BASELINE.json metric."""

from __future__ import annotations

import argparse
import importlib.util
import json
import os
import subprocess
import sys
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
                              path="fused", warmup=1, steps=2, bucket_mb=64.0, device="cuda",
                              grad_reduce_dtype="fp32", deterministic=False)
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


def _run_bench(*argv: str, env_extra: dict[str, str] | None = None) -> subprocess.CompletedProcess:
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(PYTHONPATH=str(ROOT), OMP_NUM_THREADS="2", **(env_extra or {}))
    cmd = [sys.executable, str(ROOT / "bench.py"), "--device", "cpu", "--model", "tiny", "--steps", "2",
           "--warmup", "1", "--micro-batch", "2", *argv]
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)


def _json_line(stdout: str) -> dict:
    lines = [ln for ln in stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, stdout  # rank 0 prints exactly one line
    return json.loads(lines[0])


@pytest.mark.slow
def test_bench_gpus_2_spawns_two_ranks() -> None:
    """``bench.py --gpus 2`` without a launcher starts 2 ranks itself (gloo on CPU here, RCCL on the
    GPU box) — the number it prints is a real 2-rank job, not one GPU with a warning."""
    proc = _run_bench("--gpus", "2")
    assert proc.returncode == 0, proc.stderr[-3000:]
    res = _json_line(proc.stdout)
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2"
    assert res["config"]["backend"] == "gloo"
    assert len(res["per_rank_tokens_per_sec"]) == 2 and len(res["exposed_allreduce_ms"]) == 2
    assert res["config"]["global_batch"] == 2 * 2
    assert res["value"] > 0 and res["steps"] == 2 and res["warmup"] == 1
    # a multi-rank line explains itself: RCCL transports / channels (empty on gloo) and the
    # exposed tail bucket (the tied embedding) with its queue and collective times
    assert set(res["rccl"]) >= {"transport_counts", "channels", "fallback", "env"}
    if res.get("buckets_rank0"):
        assert res["tail_bucket"]["bucket"] == res["buckets_rank0"][-1]["bucket"]
        # (queue / collective times come from GPU events: on the CPU gloo path only the payload)
        assert res["tail_bucket"]["payload_mib"] == res["buckets_rank0"][-1]["payload_mib"]


def test_bench_rejects_world_size_mismatch() -> None:
    proc = _run_bench("--gpus", "2", env_extra={"WORLD_SIZE": "1"})
    assert proc.returncode == 2
    assert "WORLD_SIZE=1" in proc.stderr


def test_bench_single_rank_cpu_contract() -> None:
    proc = _run_bench("--gpus", "1")
    assert proc.returncode == 0, proc.stderr[-3000:]
    res = _json_line(proc.stdout)
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config"):
        assert key in res
    assert res["n_gpus"] == 1 and res["higher_is_better"] is True and res["scaling"] == "weak"
