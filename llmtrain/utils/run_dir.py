"""Run directory layout: ``<root>/<run_id>/{config.yaml, meta.json, logs/, checkpoints/}``.

Reference ``utils/run_dir.py:14-45``: the run directory must not pre-exist (collisions raise),
``logs/`` is created with it (a partial directory is removed on failure) and the resolved
config is written atomically in schema order.
"""

from __future__ import annotations

import shutil
from pathlib import Path

import yaml

from llmtrain.config.schemas import RunConfig
from llmtrain.utils._atomic import atomic_write

__all__ = ["create_run_directory", "write_resolved_config"]


def create_run_directory(root_dir: str | Path, run_id: str) -> Path:
    root = Path(root_dir)
    root.mkdir(parents=True, exist_ok=True)
    run_path = root / run_id
    run_path.mkdir(exist_ok=False)
    try:
        (run_path / "logs").mkdir()
    except BaseException:
        shutil.rmtree(run_path, ignore_errors=True)
        raise
    return run_path


def write_resolved_config(run_dir: str | Path, config: RunConfig) -> Path:
    payload = config.model_dump()
    return atomic_write(
        Path(run_dir) / "config.yaml", lambda fh: yaml.safe_dump(payload, fh, sort_keys=False)
    )
