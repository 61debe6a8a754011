"""MLflow tracker (optional dependency; reference ``tracking/mlflow.py:11-87``).

``mlflow`` is imported lazily in the constructor; when it is missing a ``RuntimeError`` is
raised, which the CLI turns into a :class:`NullTracker` fallback with a warning.
"""

from __future__ import annotations

import json
from collections.abc import Mapping
from pathlib import Path
from typing import Any

__all__ = ["MLflowTracker", "_flatten_params"]


def _scalarize(value: Any) -> Any:
    if value is None:
        return "None"
    if isinstance(value, (list, tuple, set)):
        return json.dumps(list(value), default=str)
    if isinstance(value, (bool, int, float, str)):
        return value
    return str(value)


def _flatten_params(params: Mapping[str, Any], *, prefix: str = "") -> dict[str, Any]:
    """``{"a": {"b": 1}}`` → ``{"a.b": 1}``; lists become JSON, ``None`` becomes ``"None"``."""
    out: dict[str, Any] = {}
    stack: list[tuple[str, Mapping[str, Any]]] = [(prefix, params)]
    while stack:
        base, mapping = stack.pop()
        for key, value in mapping.items():
            name = f"{base}.{key}" if base else str(key)
            if isinstance(value, Mapping):
                stack.append((name, value))
            else:
                out[name] = _scalarize(value)
    return dict(sorted(out.items()))


class MLflowTracker:
    def __init__(self, *, tracking_uri: str, experiment: str, run_name: str | None = None) -> None:
        try:
            import mlflow  # type: ignore[import-not-found]
        except ModuleNotFoundError as exc:
            raise RuntimeError(
                "MLflowTracker requires the optional 'mlflow' dependency "
                "(pip install mlflow)."
            ) from exc
        self._mlflow = mlflow
        self._tracking_uri = tracking_uri
        self._experiment = experiment
        self._run_name = run_name

    def start_run(self, run_name: str | None = None, *, run_id: str | None = None) -> None:
        self._mlflow.set_tracking_uri(self._tracking_uri)
        self._mlflow.set_experiment(self._experiment)
        if run_id is not None:
            self._mlflow.start_run(run_id=run_id)
        else:
            self._mlflow.start_run(run_name=run_name or self._run_name)

    @property
    def active_run_id(self) -> str | None:
        run = self._mlflow.active_run()
        return None if run is None else run.info.run_id

    def log_params(self, params: Mapping[str, Any]) -> None:
        flat = _flatten_params(params)
        if flat:
            self._mlflow.log_params(flat)

    def log_metrics(self, metrics: Mapping[str, float], *, step: int | None = None) -> None:
        if not metrics:
            return
        values = {k: float(v) for k, v in metrics.items()}
        if step is None:
            self._mlflow.log_metrics(values)
        else:
            self._mlflow.log_metrics(values, step=step)

    def log_artifact(self, path: str | Path, *, artifact_path: str | None = None) -> None:
        self._mlflow.log_artifact(str(path), artifact_path=artifact_path)

    def end_run(self) -> None:
        self._mlflow.end_run()
