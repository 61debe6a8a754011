"""Trainer semantics (reference tests/test_trainer.py): loss decreases, LR schedule values, log /
eval cadence, tracker dependency injection, tokens/s, plus the MI355X additions (fused engine on
CPU, device-side loss accumulation, fault injection, NaN guard)."""

from __future__ import annotations

import math
from unittest.mock import Mock

import pytest

from llmtrain.config.schemas import RunConfig
from llmtrain.training import Trainer, TrainResult

from conftest import minimal_payload


def _cfg(**trainer) -> RunConfig:  # type: ignore[no-untyped-def]
    t = {"max_steps": 5, "warmup_steps": 0, "micro_batch_size": 1, "grad_accum_steps": 1}
    t.update(trainer)
    return RunConfig.model_validate(minimal_payload(trainer=t))


def _gpt_cfg(fused: bool = False, **trainer) -> RunConfig:  # type: ignore[no-untyped-def]
    t = {"max_steps": 60, "warmup_steps": 0, "micro_batch_size": 4, "grad_accum_steps": 1, "lr": 3e-3,
         "weight_decay": 0.0, "log_every_steps": 10, "eval_every_steps": 30}
    t.update(trainer)
    model = {"name": "gpt", "vocab_size": 16, "block_size": 8, "d_model": 64, "n_layers": 2, "n_heads": 2,
             "d_ff": 128, "dropout": 0.0, "extra": {"fused": fused}}
    return RunConfig.model_validate(minimal_payload(model=model, trainer=t, run={"name": "g", "seed": 123}))


def test_fit_returns_finite_result() -> None:
    cfg = _cfg()
    result = Trainer(cfg).fit()
    assert isinstance(result, TrainResult)
    assert result.final_step == 5 and math.isfinite(result.final_loss)
    assert result.total_time >= 0 and result.peak_memory == 0.0
    assert result.parameter_count and result.parameter_count == result.trainable_parameter_count


def test_dummy_loss_decreases_with_accumulation() -> None:
    result = Trainer(_cfg(max_steps=50, micro_batch_size=2, grad_accum_steps=2, lr=3e-3)).fit()
    assert result.first_step_loss is not None and result.final_loss < result.first_step_loss


@pytest.mark.parametrize("fused", [False, True])
def test_gpt_smoke_loss_decreases(fused: bool) -> None:
    trainer = Trainer(_gpt_cfg(fused=fused))
    assert (trainer.model.engine is not None) == fused
    result = trainer.fit()
    assert result.final_loss < 0.5 * (result.first_step_loss or 0)
    assert result.final_val_loss is not None and result.final_val_loss < 1.0


def test_fused_and_module_paths_agree_on_cpu() -> None:
    a = Trainer(_gpt_cfg(fused=False, max_steps=8)).fit()
    b = Trainer(_gpt_cfg(fused=True, max_steps=8)).fit()
    assert abs(a.first_step_loss - b.first_step_loss) < 1e-4  # type: ignore[operator]
    assert abs(a.final_loss - b.final_loss) < 1e-3


def test_eval_local_equals_global_without_ddp() -> None:
    trainer = Trainer(_cfg())
    local, glob = trainer._evaluate()  # type: ignore[misc]
    assert local == glob and "val/loss" in local


def test_lr_schedule_warmup_then_cosine() -> None:
    trainer = Trainer(_cfg(max_steps=10, warmup_steps=4, lr=1e-3))
    sched = trainer.scheduler
    lrs = [sched.get_last_lr()[0]]
    for _ in range(10):
        trainer.optimizer.step()
        sched.step()
        lrs.append(sched.get_last_lr()[0])
    assert lrs[0] == 0.0 and math.isclose(lrs[2], 0.5e-3) and math.isclose(lrs[4], 1e-3)
    assert math.isclose(lrs[7], 0.5e-3 * (1 + math.cos(math.pi * 0.5)), rel_tol=1e-6)
    assert lrs[10] == 0.0


def test_log_cadence_includes_final_step(trainer_records) -> None:  # type: ignore[no-untyped-def]
    Trainer(_cfg(max_steps=5, log_every_steps=2)).fit()
    steps = [r.getMessage().split()[0] for r in trainer_records if r.getMessage().startswith("step=")]
    assert steps == ["step=2/5", "step=4/5", "step=5/5"]
    line = next(r.getMessage() for r in trainer_records if r.getMessage().startswith("step=2/5"))
    assert "loss=" in line and "lr=" in line and "tokens_per_sec=" in line and "step_time=" in line


def test_eval_cadence(trainer_records) -> None:  # type: ignore[no-untyped-def]
    Trainer(_cfg(max_steps=7, eval_every_steps=3)).fit()
    evals = [r.getMessage().split()[0] for r in trainer_records if r.getMessage().startswith("val_step=")]
    assert evals == ["val_step=3/7", "val_step=6/7", "val_step=7/7"]


def test_tracker_injection_params_once_and_metric_steps() -> None:
    tracker = Mock()
    cfg = _cfg(max_steps=5, log_every_steps=2, eval_every_steps=100)
    Trainer(cfg, tracker=tracker).fit()
    tracker.log_params.assert_called_once_with(cfg.model_dump())
    train_steps = [c.kwargs["step"] for c in tracker.log_metrics.call_args_list if "train/loss" in c.args[0]]
    assert train_steps == [2, 4, 5]
    first = tracker.log_metrics.call_args_list[0].args[0]
    assert set(first) == {"train/loss", "train/lr", "train/tokens_per_sec", "train/step_time_sec", "train/tokens_total"}
    assert first["train/tokens_per_sec"] > 0 and first["train/tokens_total"] == 2 * 8


def test_fault_injection_and_nan_guard() -> None:
    with pytest.raises(RuntimeError, match="fault injection"):
        Trainer(_cfg(save_every_steps=1, extra={"fail_at_step": 2})).fit()
    Trainer(_cfg(save_every_steps=1, extra={"fail_at_step": 2, "fail_rank": 1})).fit()  # only rank 1 crashes
    # a fault before the first checkpoint would re-fire on every restart: rejected up front
    with pytest.raises(ValueError, match="fail_at_step"):
        Trainer(_cfg(save_every_steps=2, extra={"fail_at_step": 2}))
    trainer = Trainer(_cfg(lr=1e30, max_steps=3, log_every_steps=1, max_grad_norm=1e30))
    with pytest.raises(FloatingPointError):
        trainer.fit()


def test_fault_injection_fires_once_then_resume_completes(tmp_path) -> None:  # type: ignore[no-untyped-def]
    """One simulated crash per job: the run dies at ``fail_at_step``; the restarted run resumes from
    the last checkpoint and is not killed again (the K8s gang-restart e2e relies on this)."""
    cfg = _cfg(max_steps=6, save_every_steps=2, extra={"fail_at_step": 5})
    run = tmp_path / "run"
    run.mkdir()
    with pytest.raises(RuntimeError, match="fault injection"):
        Trainer(cfg, run_dir=run).fit()
    restart = tmp_path / "restart"
    restart.mkdir()
    result = Trainer(cfg, run_dir=restart).fit(resume_from=str(run / "checkpoints"))
    assert result.resumed_from_step == 4 and result.final_step == 6


def test_gpu_shape_fallback_is_opt_in() -> None:
    """On the GPU an uncovered model shape is an error unless the config opts into the module path;
    on CPU the module path is taken silently (runtime/device.py settle_fused_path)."""
    import pytest
    import torch

    from llmtrain.config.schemas import RunConfig
    from llmtrain.runtime.device import RuntimePolicy, settle_fused_path

    import yaml

    base = yaml.safe_load(open("configs/presets/gpt_smoke.yaml"))

    def cfg(extra):
        payload = dict(base, model=dict(base["model"], extra=extra))
        return RunConfig.model_validate(payload)

    gpu = RuntimePolicy(device=torch.device("cuda", 0), compute_dtype=torch.bfloat16, use_fused=True)
    with pytest.raises(ValueError, match="allow_module_fallback"):
        settle_fused_path(gpu, cfg({}), supported=False)
    assert not settle_fused_path(gpu, cfg({"allow_module_fallback": True}), supported=False).use_fused
    assert settle_fused_path(gpu, cfg({}), supported=True).use_fused
    cpu = RuntimePolicy(device=torch.device("cpu"), compute_dtype=torch.float32, use_fused=True)
    assert not settle_fused_path(cpu, cfg({}), supported=False).use_fused


def test_cuda_graph_requirements_are_checked() -> None:
    """trainer.extra.cuda_graph (llmtrain.training.graph_step): every unmet requirement of a
    captured step is a config error naming it, not a silent eager run."""
    import torch

    from llmtrain.training.graph_step import check_graphable
    from llmtrain.training.optim import FusedAdamW

    class _FakeFused(FusedAdamW):  # isinstance check only
        def __init__(self) -> None:  # noqa: D107 - no store needed
            pass

    ok = dict(device=torch.device("cuda"), fused=True, optimizer=_FakeFused(), ddp_active=False)
    check_graphable(**ok)
    for key, bad, word in [
        ("device", torch.device("cpu"), "GPU"),
        ("fused", False, "fused engine"),
        ("optimizer", object(), "fused AdamW"),
        ("ddp_active", True, "single-process"),
    ]:
        with pytest.raises(ValueError, match=word):
            check_graphable(**{**ok, key: bad})
