"""Launcher helpers for the K8s entrypoint (``k8s/entrypoint.sh``), testable in Python.

    python -m llmtrain.launch latest-checkpoint --runs-root /app/runs --run-id llmtrain
    python -m llmtrain.launch restart-tag

``latest-checkpoint`` prints the newest ``step_*.pt`` of a job across its run directories — the
original ``<run_id>`` and every gang restart's ``<run_id>-restart-<tag>`` — or nothing (exit 1)
when there is none; "newest" is the highest step, the most recently written file on a tie.
A half-written file never matches: checkpoints are written to ``*.pt.tmp`` and renamed
(training/checkpoint.py).  ``restart-tag`` prints a run-id suffix that every pod of ONE Job
incarnation shares (the Job's UID, which the Job controller puts on each pod as the
``batch.kubernetes.io/controller-uid`` label and the manifest passes in as ``JOB_UID``), so the
ranks of a restarted gang agree on their new ``--run-id`` — a per-pod ``date`` did not
(reference entrypoint: ``k8s/entrypoint.sh:20-89``).
"""

from __future__ import annotations

import argparse
import os
import re
import sys
from pathlib import Path

__all__ = ["latest_checkpoint", "restart_tag"]

_STEP = re.compile(r"^step_(\d+)\.pt$")


def _job_dirs(runs_root: Path, run_id: str) -> list[Path]:
    if not runs_root.is_dir():
        return []
    prefix = f"{run_id}-restart-"
    return [d for d in runs_root.iterdir() if d.is_dir() and (d.name == run_id or d.name.startswith(prefix))]


def latest_checkpoint(runs_root: str | os.PathLike[str], run_id: str) -> Path | None:
    best: tuple[int, float, str] | None = None
    best_path: Path | None = None
    for run_dir in _job_dirs(Path(runs_root), run_id):
        ckpts = run_dir / "checkpoints"
        if not ckpts.is_dir():
            continue
        for f in ckpts.iterdir():
            m = _STEP.match(f.name)
            if not m or not f.is_file():
                continue
            key = (int(m.group(1)), f.stat().st_mtime, f.name)
            if best is None or key > best:
                best, best_path = key, f
    return best_path


def restart_tag(env: dict[str, str] | None = None) -> str:
    env = dict(os.environ) if env is None else env
    uid = env.get("JOB_UID") or env.get("RESTART_TAG")
    if not uid:
        raise RuntimeError("JOB_UID (the Job's controller-uid label) is not set; every rank must share the tag")
    return re.sub(r"[^a-z0-9]", "", uid.lower())[:12] or "0"


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(prog="python -m llmtrain.launch")
    sub = ap.add_subparsers(dest="cmd", required=True)
    lc = sub.add_parser("latest-checkpoint")
    lc.add_argument("--runs-root", required=True)
    lc.add_argument("--run-id", required=True)
    sub.add_parser("restart-tag")
    args = ap.parse_args(argv)
    if args.cmd == "latest-checkpoint":
        path = latest_checkpoint(args.runs_root, args.run_id)
        if path is None:
            return 1
        print(path)
        return 0
    print(restart_tag())
    return 0


if __name__ == "__main__":
    sys.exit(main())
