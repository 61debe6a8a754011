"""Tracking contract (reference tests/test_tracking.py): NullTracker, MLflow call contract with
a fake ``mlflow`` module, parameter flattening, and mlflow staying optional."""

from __future__ import annotations

import sys
import types
from pathlib import Path

import pytest

from llmtrain.tracking import MLflowTracker, NullTracker, Tracker
from llmtrain.tracking.mlflow import _flatten_params


def test_null_tracker_is_tracker() -> None:
    t = NullTracker()
    assert isinstance(t, Tracker)
    t.start_run("x")
    t.log_params({"a": 1})
    t.log_metrics({"m": 1.0}, step=1)
    t.log_artifact(Path("x"), artifact_path="a")
    t.end_run()


def test_mlflow_call_contract(monkeypatch: pytest.MonkeyPatch) -> None:
    calls: list[tuple] = []
    fake = types.ModuleType("mlflow")
    for name in ("set_tracking_uri", "set_experiment", "start_run", "log_params", "log_metrics", "log_artifact", "end_run"):
        setattr(fake, name, lambda *a, _n=name, **k: calls.append((_n, a, k)))
    fake.active_run = lambda: types.SimpleNamespace(info=types.SimpleNamespace(run_id="abc"))
    monkeypatch.setitem(sys.modules, "mlflow", fake)
    t = MLflowTracker(tracking_uri="sqlite:///x.db", experiment="exp", run_name="rn")
    t.start_run()
    t.log_params({"model": {"d": 1, "l": [1, 2]}, "x": None})
    t.log_metrics({"train/loss": 1}, step=3)
    t.log_metrics({})
    t.log_artifact("f.yaml", artifact_path="artifacts")
    t.end_run()
    names = [c[0] for c in calls]
    assert names == ["set_tracking_uri", "set_experiment", "start_run", "log_params", "log_metrics", "log_artifact", "end_run"]
    assert calls[2][2] == {"run_name": "rn"}
    assert calls[3][1][0] == {"model.d": 1, "model.l": "[1, 2]", "x": "None"}
    assert calls[4][1][0] == {"train/loss": 1.0} and calls[4][2] == {"step": 3}
    assert t.active_run_id == "abc"


def test_flatten() -> None:
    assert _flatten_params({"a": {"b": {"c": 1}}, "t": (1, "x"), "o": object}) ["a.b.c"] == 1
    flat = _flatten_params({"s": {1, }, "f": 1.5, "b": True})
    assert flat == {"b": True, "f": 1.5, "s": "[1]"}


def test_mlflow_is_optional(monkeypatch: pytest.MonkeyPatch) -> None:
    monkeypatch.setitem(sys.modules, "mlflow", None)
    with pytest.raises(RuntimeError, match="optional 'mlflow'"):
        MLflowTracker(tracking_uri="x", experiment="y")


def test_real_mlflow_sqlite(tmp_path: Path) -> None:
    mlflow = pytest.importorskip("mlflow")
    t = MLflowTracker(tracking_uri=f"sqlite:///{tmp_path / 'm.db'}", experiment="e")
    t.start_run("r")
    t.log_metrics({"x": 1.0}, step=1)
    t.end_run()
    assert mlflow is not None
