"""Atomic file writes: write to ``<name>.tmp`` in the same directory, then ``os.replace``."""

from __future__ import annotations

import os
from collections.abc import Callable
from pathlib import Path
from typing import IO


def atomic_write(path: Path, writer: Callable[[IO[str]], None]) -> Path:
    tmp = path.with_name(path.name + ".tmp")
    with tmp.open("w", encoding="utf-8") as handle:
        writer(handle)
        handle.flush()
        os.fsync(handle.fileno())
    os.replace(tmp, path)
    return path
