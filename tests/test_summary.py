"""Run summary formats (reference tests/test_summary.py)."""

from __future__ import annotations

from pathlib import Path

import pytest

from llmtrain.config.schemas import RunConfig
from llmtrain.training.trainer import TrainResult
from llmtrain.utils.summary import format_run_summary

from conftest import minimal_payload


def _cfg() -> RunConfig:
    return RunConfig.model_validate(minimal_payload())


def _result(**kw) -> TrainResult:  # type: ignore[no-untyped-def]
    base = dict(final_step=5, final_loss=1.25, final_val_loss=None, total_time=2.5, peak_memory=0.0)
    base.update(kw)
    return TrainResult(**base)


def test_json_keys(monkeypatch: pytest.MonkeyPatch) -> None:
    monkeypatch.setenv("RANK", "0")
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    s = format_run_summary(config=_cfg(), run_id="rid", run_dir=Path("runs/rid"), json_output=True)
    assert isinstance(s, dict)
    assert set(s) == {"run_id", "output_dir", "model", "data", "trainer", "ddp", "mlflow"}
    assert s["ddp"]["env"]["RANK"] == "0" and s["ddp"]["env"]["WORLD_SIZE"] is None
    assert set(s["model"]) == {
        "name", "init", "block_size", "d_model", "n_layers", "n_heads", "d_ff", "dropout",
        "tie_embeddings", "vocab_size",
    }
    assert len(s["trainer"]) == 10 and len(s["data"]) == 8 and len(s["mlflow"]) == 5


def test_json_training_block_optional_fields() -> None:
    s = format_run_summary(
        config=_cfg(), run_id="r", run_dir="runs/r", json_output=True,
        train_result=_result(parameter_count=10, trainable_parameter_count=9, final_val_loss=1.5,
                             val_metrics={"val/loss": 1.5}, first_step_loss=3.0, resumed_from_step=2),
        resumed_from="prev",
    )
    t = s["training"]
    assert t["final_step"] == 5 and t["parameter_count"] == 10 and t["trainable_parameter_count"] == 9
    assert t["final_val_loss"] == 1.5 and t["val_metrics"] == {"val/loss": 1.5}
    assert t["resumed_from_step"] == 2 and s["resumed_from"] == "prev"
    bare = format_run_summary(config=_cfg(), run_id="r", run_dir="runs/r", json_output=True, train_result=_result())
    assert "resumed_from" not in bare and "final_val_loss" not in bare["training"]
    assert bare["training"]["first_step_loss"] is None


def test_dry_run_fields() -> None:
    s = format_run_summary(
        config=_cfg(), run_id="r", run_dir="runs/r", json_output=True,
        resolved_model_adapter="dummy_gpt", resolved_data_module="dummy_text", dry_run_steps_executed=5,
    )
    assert s["resolved_model_adapter"] == "dummy_gpt" and s["dry_run_steps_executed"] == 5


def test_text_format() -> None:
    text = format_run_summary(
        config=_cfg(), run_id="rid", run_dir="runs/rid",
        train_result=_result(parameter_count=7, final_val_loss=1.5, val_metrics={"val/loss": 1.5}),
        resumed_from="x",
    )
    assert isinstance(text, str)
    lines = text.splitlines()
    assert lines[0] == "Planned run:"
    assert lines[1] == "  Run ID: rid"
    assert any(line.startswith("  Model: name=dummy_gpt") for line in lines)
    assert any("env=[RANK=" in line for line in lines)
    assert "  Resumed from: x" in lines
    training = next(line for line in lines if line.startswith("  Training:"))
    assert "final_loss=1.2500" in training and "parameter_count=7" in training and "final_val_loss=1.5000" in training
    assert lines[-1] == "  Validation: val/loss=1.5000"


def test_text_dry_run_line() -> None:
    text = format_run_summary(config=_cfg(), run_id="r", run_dir="runs/r", dry_run_steps_executed=3)
    assert "  Dry run: resolved_model_adapter=None resolved_data_module=None steps_executed=3" in text
