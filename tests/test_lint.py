"""``make lint``'s built-in checker (scripts/lint.py) passes on the tree: every module compiles, no
unused imports, line limits, and no CUDA compatibility layers in the HIP sources."""

from __future__ import annotations

import subprocess
import sys

from conftest import REPO


def test_builtin_lint_clean() -> None:
    proc = subprocess.run([sys.executable, str(REPO / "scripts" / "lint.py"), "--builtin-only"], cwd=REPO,
                          capture_output=True, text=True, timeout=120)
    assert proc.returncode == 0, proc.stdout[-3000:]
