"""Run ids (reference tests/test_run_id.py): slug rules, format, nogit fallback, collisions."""

from __future__ import annotations

import re
import subprocess
from pathlib import Path

import pytest

from llmtrain.utils import run_id as run_id_mod
from llmtrain.utils.run_id import generate_run_id, slugify_run_name


@pytest.mark.parametrize(
    "name,slug",
    [
        ("My Run", "my_run"),
        ("  --Weird!!Name__  ", "weird_name"),
        ("a" * 60, "a" * 40),
        ("!!!", "run"),
        ("gpt2-124m mi355x", "gpt2-124m_mi355x"),
        ("x--y", "x_y"),
    ],
)
def test_slugify(name: str, slug: str) -> None:
    assert slugify_run_name(name) == slug


def test_format_with_git(monkeypatch: pytest.MonkeyPatch) -> None:
    monkeypatch.setattr(run_id_mod, "_get_short_git_sha", lambda: "abc123")
    rid = generate_run_id("My Run")
    assert re.fullmatch(r"\d{8}_\d{6}_abc123_my_run", rid)


def test_nogit_fallback(monkeypatch: pytest.MonkeyPatch) -> None:
    def boom(*a, **k):  # type: ignore[no-untyped-def]
        raise FileNotFoundError("git")

    monkeypatch.setattr(subprocess, "run", boom)
    assert run_id_mod._get_short_git_sha() == "nogit"

    def fail(*a, **k):  # type: ignore[no-untyped-def]
        raise subprocess.CalledProcessError(128, "git")

    monkeypatch.setattr(subprocess, "run", fail)
    assert run_id_mod._get_short_git_sha() == "nogit"


def test_collision_suffixes(tmp_path: Path, monkeypatch: pytest.MonkeyPatch) -> None:
    monkeypatch.setattr(run_id_mod, "_get_short_git_sha", lambda: "sha")
    base = run_id_mod._append_collision_suffix("rid", tmp_path)
    assert base == "rid"
    (tmp_path / "rid").mkdir()
    assert run_id_mod._append_collision_suffix("rid", tmp_path) == "rid__01"
    for i in range(1, 100):
        (tmp_path / f"rid__{i:02d}").mkdir()
    with pytest.raises(RuntimeError, match="collision limit"):
        run_id_mod._append_collision_suffix("rid", tmp_path)
