"""CLI end-to-end (reference tests/test_cli.py): help, validate/print-config (text + JSON,
exit 2 on errors), dry run, full training runs (JSON / text), resume, tracker fallback and
lifecycle, wiring with mocked collaborators."""

from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path
from unittest.mock import Mock

import pytest
import yaml

from llmtrain import cli as cli_mod
from llmtrain.cli import main

from conftest import REPO, minimal_payload

GPT_SMOKE = REPO / "configs" / "presets" / "gpt_smoke.yaml"


def _write(tmp: Path, **over) -> Path:  # type: ignore[no-untyped-def]
    path = tmp / "cfg.yaml"
    path.write_text(yaml.safe_dump(minimal_payload(**over)), encoding="utf-8")
    return path


def _run(*args: str, cwd: Path) -> subprocess.CompletedProcess[str]:
    env = dict(os.environ, PYTHONPATH=str(REPO))
    return subprocess.run(
        [sys.executable, "-m", "llmtrain", *args], cwd=cwd, env=env, capture_output=True, text=True, timeout=300
    )


def test_help_and_version(in_tmp: Path) -> None:
    proc = _run("--help", cwd=in_tmp)
    assert proc.returncode == 0 and "train" in proc.stdout and "print-config" in proc.stdout
    assert _run("--version", cwd=in_tmp).stdout.startswith("llmtrain ")


def test_validate_ok_and_error(in_tmp: Path, capsys: pytest.CaptureFixture[str]) -> None:
    good = _write(in_tmp)
    assert main(["validate", "--config", str(good)]) == 0
    assert "Config validation succeeded." in capsys.readouterr().out
    assert main(["validate", "--config", str(good), "--json"]) == 0
    assert json.loads(capsys.readouterr().out) == {"status": "ok"}
    bad = _write(in_tmp, model={"name": "m", "d_model": 384, "n_heads": 7})
    assert main(["validate", "--config", str(bad), "--json"]) == 2
    err = json.loads(capsys.readouterr().err)
    assert err["status"] == "error" and err["errors"] and "validation failed" in err["message"]
    assert main(["validate", "--config", str(bad)]) == 2
    assert "Config error:" in capsys.readouterr().err


def test_print_config(in_tmp: Path, capsys: pytest.CaptureFixture[str]) -> None:
    path = _write(in_tmp)
    assert main(["print-config", "--config", str(path), "--json"]) == 0
    data = json.loads(capsys.readouterr().out)
    assert data["trainer"]["lr"] == 3e-4 and data["model"]["name"] == "dummy_gpt"
    assert main(["print-config", "--config", str(path)]) == 0
    assert yaml.safe_load(capsys.readouterr().out)["run"]["seed"] == 1337


def test_dry_run_json(in_tmp: Path, capsys: pytest.CaptureFixture[str]) -> None:
    path = _write(in_tmp)
    assert main(["train", "--config", str(path), "--dry-run", "--json", "--run-id", "dry"]) == 0
    out = json.loads(capsys.readouterr().out)
    assert out["dry_run_steps_executed"] == 5 and out["resolved_model_adapter"] == "dummy_gpt"
    run_dir = in_tmp / "runs" / "dry"
    assert (run_dir / "config.yaml").exists() and (run_dir / "meta.json").exists()


def test_full_run_json_and_text(in_tmp: Path, capsys: pytest.CaptureFixture[str]) -> None:
    path = _write(in_tmp)
    assert main(["train", "--config", str(path), "--json", "--run-id", "j"]) == 0
    captured = capsys.readouterr()
    out = json.loads(captured.out)  # stdout carries exactly one JSON document
    assert out["training"]["final_step"] == 5 and out["run_id"] == "j"
    assert main(["train", "--config", str(path), "--run-id", "t"]) == 0
    text = capsys.readouterr().out
    assert "Planned run:" in text and "Training: final_step=5" in text
    ckpts = sorted((in_tmp / "runs" / "t" / "checkpoints").glob("step_*.pt"))
    assert [p.name for p in ckpts] == ["step_000005.pt"]


def test_unknown_plugin_exit_2(in_tmp: Path, capsys: pytest.CaptureFixture[str]) -> None:
    path = _write(in_tmp, model={"name": "no_such_model"})
    assert main(["train", "--config", str(path), "--json"]) == 2
    assert "Unknown model adapter" in capsys.readouterr().err


def test_gpt_smoke_preset_subprocess(in_tmp: Path) -> None:
    cfg = yaml.safe_load(GPT_SMOKE.read_text())
    cfg["trainer"]["max_steps"] = 20
    cfg["mlflow"]["enabled"] = False
    path = in_tmp / "gpt.yaml"
    path.write_text(yaml.safe_dump(cfg))
    proc = _run("train", "--config", str(path), "--json", cwd=in_tmp)
    assert proc.returncode == 0, proc.stderr
    out = json.loads(proc.stdout)
    assert out["training"]["final_step"] == 20
    assert out["training"]["final_loss"] < out["training"]["first_step_loss"]
    assert "step=20/20" in proc.stderr  # trainer logs routed to stderr in --json mode


def test_resume_via_cli(in_tmp: Path, capsys: pytest.CaptureFixture[str]) -> None:
    path = _write(in_tmp, trainer={"max_steps": 4, "warmup_steps": 0, "micro_batch_size": 1, "save_every_steps": 2})
    assert main(["train", "--config", str(path), "--json", "--run-id", "first"]) == 0
    capsys.readouterr()
    ckpt_dir = in_tmp / "runs" / "first" / "checkpoints"
    for spec in (str(ckpt_dir), str(ckpt_dir / "step_000004.pt"), "first"):
        assert main(["train", "--config", str(path), "--json", "--resume", spec]) == 0
        out = json.loads(capsys.readouterr().out)
        assert out["resumed_from"] == spec and out["training"]["resumed_from_step"] == 4
    assert main(["train", "--config", str(path), "--resume", "missing_run"]) == 1
    assert "Training failed" in capsys.readouterr().err


def test_mlflow_missing_falls_back(in_tmp: Path, monkeypatch: pytest.MonkeyPatch, capsys: pytest.CaptureFixture[str]) -> None:
    monkeypatch.setitem(sys.modules, "mlflow", None)
    path = _write(in_tmp, mlflow={"enabled": True, "tracking_uri": "sqlite:///x.db"})
    assert main(["train", "--config", str(path), "--json"]) == 0
    assert "falling back to NullTracker" in capsys.readouterr().err


def test_handle_train_wiring_and_tracker_always_ended(in_tmp: Path, monkeypatch: pytest.MonkeyPatch,
                                                      capsys: pytest.CaptureFixture[str]) -> None:
    tracker = Mock()
    trainer_cls = Mock()
    trainer_cls.return_value.fit.side_effect = RuntimeError("boom")
    monkeypatch.setattr(cli_mod, "_create_tracker", lambda cfg, logger: tracker)
    monkeypatch.setattr(cli_mod, "Trainer", trainer_cls)
    path = _write(in_tmp, mlflow={"enabled": True, "run_name": "rn"})
    assert main(["train", "--config", str(path), "--run-id", "w", "--resume", "r0"]) == 1
    assert "Training failed: boom" in capsys.readouterr().err
    tracker.start_run.assert_called_once_with(run_name="rn")
    tracker.end_run.assert_called_once()
    kwargs = trainer_cls.call_args.kwargs
    assert kwargs["tracker"] is tracker and kwargs["ddp_state"] is None
    assert kwargs["run_dir"] == Path("runs") / "w"
    trainer_cls.return_value.fit.assert_called_once_with(resume_from="r0")
