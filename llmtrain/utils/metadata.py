"""``meta.json`` for a run directory (reference ``utils/metadata.py:15-81``)."""

from __future__ import annotations

import json
import os
import platform
import subprocess
import sys
from datetime import datetime, timezone
from pathlib import Path
from typing import Any

from llmtrain.utils._atomic import atomic_write

__all__ = ["DDP_ENV_KEYS", "generate_meta", "write_meta_json"]

DDP_ENV_KEYS = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")


def _get_git_sha() -> str | None:
    try:
        out = subprocess.run(
            ["git", "rev-parse", "HEAD"], check=True, capture_output=True, text=True, timeout=10
        )
    except (subprocess.CalledProcessError, FileNotFoundError, subprocess.TimeoutExpired):
        return "nogit"
    return out.stdout.strip() or None


def _utc_now_z() -> str:
    return datetime.now(timezone.utc).replace(microsecond=0).strftime("%Y-%m-%dT%H:%M:%SZ")


def generate_meta(
    *,
    run_id: str,
    run_name: str,
    config_path: str | None,
    resolved_config_path: str | None,
) -> dict[str, Any]:
    return {
        "meta_version": 1,
        "run_id": run_id,
        "run_name": run_name,
        "created_at": _utc_now_z(),
        "git_sha": _get_git_sha(),
        "python_version": platform.python_version(),
        "platform": platform.platform(),
        "argv": list(sys.argv),
        "cwd": os.getcwd(),
        "config_path": config_path,
        "resolved_config_path": resolved_config_path,
        "ddp_env": {key: (os.environ.get(key) or None) for key in DDP_ENV_KEYS},
        "hostname": platform.node(),
        "pid": os.getpid(),
    }


def write_meta_json(run_dir: str | Path, meta: dict[str, Any]) -> Path:
    def _dump(handle) -> None:  # type: ignore[no-untyped-def]
        json.dump(meta, handle, ensure_ascii=False, indent=2)
        handle.write("\n")

    return atomic_write(Path(run_dir) / "meta.json", _dump)
