"""Single-process "fake world" checks of the Trainer's rank-dependent branches (reference
``tests/test_distributed.py:236-694``): a real 1-process gloo group stands in for the world while
the ``DDPState`` claims rank r of 2 and the metric collectives are replaced by a two-identical-ranks
simulation.  Complements the real 2-process tests in ``test_distributed.py`` with the rank != 0
paths that a 2-process run only covers implicitly:

* wrapping: ``world_size > 1`` wraps (torch DDP for ``dummy_gpt``, the flat-buffer reducer for the
  fused GPT), ``world_size == 1`` / no state does not, ``_raw_model`` unwraps;
* rank-0-only I/O: tracker params/metrics and checkpoint files only on rank 0, none on rank 1;
* metric names: ``train/*_rank_{r}`` + global ``train/*`` under DDP, no suffix without it;
* ``_gather_scalars`` / ``_reduce_metrics`` semantics.
"""

from __future__ import annotations

import socket
from pathlib import Path
from unittest.mock import Mock

import pytest
import torch
import torch.distributed as dist
from torch.nn.parallel import DistributedDataParallel

from llmtrain.config.schemas import RunConfig
from llmtrain.parallel.dist import DDPState
from llmtrain.parallel.reducer import FlatDataParallel
from llmtrain.training.trainer import Trainer

from conftest import minimal_payload

WORLD = 2


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def one_process_group(monkeypatch: pytest.MonkeyPatch):
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    yield
    dist.destroy_process_group()


@pytest.fixture
def two_identical_ranks(one_process_group, monkeypatch: pytest.MonkeyPatch):
    """Metric collectives as if a second rank held exactly this rank's values."""

    def all_gather(out: list[torch.Tensor], local: torch.Tensor, *a, **k) -> None:
        for t in out:
            t.copy_(local)

    real_all_reduce = dist.all_reduce

    def all_reduce(t: torch.Tensor, op=dist.ReduceOp.SUM, group=None, async_op=False):  # type: ignore[no-untyped-def]
        if async_op:  # gradient buckets: the real (1-process) collective, an identity
            return real_all_reduce(t, op=op, group=group, async_op=True)
        if op == dist.ReduceOp.SUM:
            t.mul_(WORLD)
        # MAX / MIN (replica checksums) of identical ranks: unchanged
        return None

    monkeypatch.setattr(dist, "all_gather", all_gather)
    monkeypatch.setattr(dist, "all_reduce", all_reduce)


def _cfg(model: str = "dummy_gpt", steps: int = 4, **trainer: object) -> RunConfig:
    tr = {"max_steps": steps, "warmup_steps": 0, "micro_batch_size": 2, "grad_accum_steps": 1,
          "log_every_steps": 2, "eval_every_steps": steps, "save_every_steps": 2}
    tr.update(trainer)
    m: dict[str, object] = {"name": model}
    if model == "gpt":
        m.update(vocab_size=32, block_size=8, d_model=64, n_layers=1, n_heads=2, d_ff=64, dropout=0.0,
                 extra={"fused": True})
    return RunConfig.model_validate(minimal_payload(model=m, trainer=tr, ddp={"enabled": True}))


def _logged_keys(tracker: Mock) -> set[str]:
    keys: set[str] = set()
    for call in tracker.log_metrics.call_args_list:
        keys |= set(call.args[0])
    return keys


# -- wrapping ---------------------------------------------------------------------------------


@pytest.mark.parametrize("model,wrapper", [("dummy_gpt", DistributedDataParallel), ("gpt", FlatDataParallel)])
def test_wrapped_when_world_gt_1_and_raw_model_unwraps(one_process_group, model, wrapper) -> None:
    tr = Trainer(_cfg(model), ddp_state=DDPState(0, WORLD, 0, True))
    assert isinstance(tr.model, wrapper)
    assert tr._raw_model is tr.model.module
    assert not isinstance(tr._raw_model, (DistributedDataParallel, FlatDataParallel))


def test_not_wrapped_for_world_1_or_no_state(one_process_group) -> None:
    assert not isinstance(Trainer(_cfg(), ddp_state=DDPState(0, 1, 0, True)).model, DistributedDataParallel)
    tr = Trainer(_cfg(), ddp_state=None)
    assert not isinstance(tr.model, DistributedDataParallel)
    assert tr._raw_model is tr.model


# -- rank-0-only I/O ---------------------------------------------------------------------------


@pytest.mark.parametrize("model", ["dummy_gpt", "gpt"])
def test_rank1_never_touches_tracker_or_checkpoints(two_identical_ranks, tmp_path: Path, model: str) -> None:
    tracker = Mock()
    run_dir = tmp_path / "rank1"
    run_dir.mkdir()
    result = Trainer(_cfg(model), run_dir=run_dir, tracker=tracker, ddp_state=DDPState(1, WORLD, 1, False)).fit()
    tracker.log_params.assert_not_called()
    tracker.log_metrics.assert_not_called()
    assert list((run_dir / "checkpoints").glob("step_*.pt")) == [] if (run_dir / "checkpoints").exists() else True
    assert result.final_step == 4 and result.final_val_loss is not None  # rank 1 still evaluates


@pytest.mark.parametrize("model", ["dummy_gpt", "gpt"])
def test_rank0_logs_and_checkpoints(two_identical_ranks, tmp_path: Path, model: str) -> None:
    tracker = Mock()
    run_dir = tmp_path / "rank0"
    run_dir.mkdir()
    Trainer(_cfg(model), run_dir=run_dir, tracker=tracker, ddp_state=DDPState(0, WORLD, 0, True)).fit()
    tracker.log_params.assert_called_once()
    assert sorted(p.name for p in (run_dir / "checkpoints").glob("step_*.pt")) == ["step_000002.pt", "step_000004.pt"]
    keys = _logged_keys(tracker)
    for r in range(WORLD):
        for name in ("loss", "lr", "tokens_per_sec", "step_time_sec", "tokens_total", "allreduce_ms"):
            assert f"train/{name}_rank_{r}" in keys
        assert f"val/loss_rank_{r}" in keys
    assert {"train/loss", "train/lr", "train/tokens_per_sec", "train/tokens_total", "train/step_time_sec",
            "train/allreduce_ms", "val/loss"} <= keys


# -- metric names and values -------------------------------------------------------------------


def test_no_rank_suffix_without_ddp(tmp_path: Path) -> None:
    tracker = Mock()
    cfg = RunConfig.model_validate(minimal_payload(trainer={
        "max_steps": 2, "warmup_steps": 0, "micro_batch_size": 2, "grad_accum_steps": 1, "log_every_steps": 1}))
    Trainer(cfg, tracker=tracker).fit()
    keys = _logged_keys(tracker)
    assert "train/loss" in keys and not any("_rank_" in k for k in keys)


def test_global_tokens_are_the_sum_over_ranks(two_identical_ranks) -> None:
    tracker = Mock()
    Trainer(_cfg(steps=2), tracker=tracker, ddp_state=DDPState(0, WORLD, 0, True)).fit()
    last = {}
    for call in tracker.log_metrics.call_args_list:
        last.update(call.args[0])
    per_rank = last["train/tokens_total_rank_0"]
    assert last["train/tokens_total"] == WORLD * per_rank > 0
    assert last["train/loss"] == pytest.approx(last["train/loss_rank_0"])  # identical ranks: same mean


def test_gather_and_reduce_helpers(two_identical_ranks) -> None:
    main = Trainer(_cfg(), ddp_state=DDPState(0, WORLD, 0, True))
    other = Trainer(_cfg(), ddp_state=DDPState(1, WORLD, 1, False))
    rows = main._gather_scalars(a=1.5, b=2.0)
    assert rows == [{"a": 1.5, "b": 2.0}] * WORLD
    assert other._gather_scalars(a=1.5) is None
    assert main._reduce_metrics(x=3.0) == {"x": 3.0 * WORLD}
    solo = Trainer(_cfg(), ddp_state=None)
    assert solo._reduce_metrics(x=3.0) == {"x": 3.0}
    assert solo._gather_scalars(x=3.0) == [{"x": 3.0}]
