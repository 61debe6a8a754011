"""Run IDs: ``{UTC %Y%m%d_%H%M%S}_{short git sha | nogit}_{slug}`` (reference ``utils/run_id.py``).

Slug rules: lower-case, runs of characters outside ``[a-z0-9-_]`` become ``_``, leading and
trailing ``-``/``_`` trimmed, repeated separators collapsed to ``_``, at most 40 characters,
``"run"`` when nothing is left. An existing directory gets ``__01`` … ``__99``.
"""

from __future__ import annotations

import re
import subprocess
from datetime import datetime, timezone
from pathlib import Path

__all__ = ["generate_run_id", "slugify_run_name"]

_NOT_SLUG = re.compile(r"[^a-z0-9\-_]+")
_SEP_RUN = re.compile(r"[-_]{2,}")
_MAX_SLUG = 40
_MAX_SUFFIX = 99


def _get_short_git_sha() -> str:
    try:
        out = subprocess.run(
            ["git", "rev-parse", "--short", "HEAD"],
            check=True,
            capture_output=True,
            text=True,
            timeout=10,
        )
    except (subprocess.CalledProcessError, FileNotFoundError, subprocess.TimeoutExpired):
        return "nogit"
    return out.stdout.strip() or "nogit"


def slugify_run_name(name: str) -> str:
    slug = _NOT_SLUG.sub("_", name.strip().lower()).strip("-_")
    slug = _SEP_RUN.sub("_", slug)
    return slug[:_MAX_SLUG] if slug else "run"


def _append_collision_suffix(run_id: str, root_dir: Path) -> str:
    if not (root_dir / run_id).exists():
        return run_id
    for n in range(1, _MAX_SUFFIX + 1):
        candidate = f"{run_id}__{n:02d}"
        if not (root_dir / candidate).exists():
            return candidate
    raise RuntimeError("Run ID collision limit reached (tried __01 through __99).")


def generate_run_id(run_name: str, root_dir: str | Path | None = None) -> str:
    stamp = datetime.now(timezone.utc).strftime("%Y%m%d_%H%M%S")
    run_id = f"{stamp}_{_get_short_git_sha()}_{slugify_run_name(run_name)}"
    return run_id if root_dir is None else _append_collision_suffix(run_id, Path(root_dir))
