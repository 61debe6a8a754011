"""Tracker protocol and the no-op tracker (reference ``tracking/base.py:10-48``)."""

from __future__ import annotations

from collections.abc import Mapping
from pathlib import Path
from typing import Any, Protocol, runtime_checkable

__all__ = ["NullTracker", "Tracker"]


@runtime_checkable
class Tracker(Protocol):
    def start_run(self, run_name: str | None = None, *, run_id: str | None = None) -> None: ...

    def log_params(self, params: Mapping[str, Any]) -> None: ...

    def log_metrics(self, metrics: Mapping[str, float], *, step: int | None = None) -> None: ...

    def log_artifact(self, path: str | Path, *, artifact_path: str | None = None) -> None: ...

    def end_run(self) -> None: ...


class NullTracker:
    """Accepts every call and records nothing."""

    def start_run(self, run_name: str | None = None, *, run_id: str | None = None) -> None:
        return None

    def log_params(self, params: Mapping[str, Any]) -> None:
        return None

    def log_metrics(self, metrics: Mapping[str, float], *, step: int | None = None) -> None:
        return None

    def log_artifact(self, path: str | Path, *, artifact_path: str | None = None) -> None:
        return None

    def end_run(self) -> None:
        return None
