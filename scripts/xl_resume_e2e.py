#!/usr/bin/env python3
"""GPT-2 XL 1.5B end to end through the real CLI on the GPU (BASELINE config 5 on one MI355X):
``torchrun`` + RCCL (world 1), gradient accumulation, checkpoints, an injected crash mid-run and
``--resume``; the resumed run must end exactly where the uninterrupted one does.

    python scripts/xl_resume_e2e.py [OUT_DIR]

Run A trains steps 1..6 uninterrupted.  Run B is the same config with ``fail_at_step: 5``: it
checkpoints at step 4, dies in step 5, and is resumed from its run id to finish steps 5..6.  Both
run with ``run.deterministic: true``, so the final losses must agree to <= 1e-5 (the reference's
resume tolerance, tests/test_checkpoint.py:301-320).  Prints one JSON line.
"""

from __future__ import annotations

import json
import os
import shutil
import subprocess
import sys
import time
from pathlib import Path

import yaml

REPO = Path(__file__).resolve().parents[1]
# the 18.7 GB checkpoints go to scratch space outside the repository (never into gpurun_out/)
RUNS = Path(os.environ.get("TMPDIR", "/tmp")) / "llmtrain_xl_e2e_runs"


def _config(out: Path, name: str, fail_at: int | None) -> Path:
    cfg = yaml.safe_load((REPO / "configs/presets/gpt2_xl_mi355x_ddp8.yaml").read_text())
    cfg["run"]["name"] = name
    # the preset's own micro-batch x grad-accum (32 x 2 since round 5)
    cfg["trainer"].update(max_steps=6, save_every_steps=4, log_every_steps=1, eval_every_steps=1000, warmup_steps=2)
    cfg["trainer"]["extra"] = {"keep_last_k": 1, "bucket_cap_mb": 128}
    if fail_at is not None:
        cfg["trainer"]["extra"]["fail_at_step"] = fail_at
    cfg["data"]["extra"] = {"train_sequences": 512, "val_sequences": 32, "branching": 4}
    cfg["output"]["root_dir"] = str(RUNS)
    cfg["logging"]["log_to_file"] = False
    path = out / f"{name}.yaml"
    path.write_text(yaml.safe_dump(cfg))
    return path


def _train(cfg: Path, run_id: str, resume: str | None, log: Path) -> tuple[int, dict | None]:
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(29400 + (os.getpid() % 500)),
           "-m", "llmtrain", "train", "--config", str(cfg), "--json", "--run-id", run_id]
    if resume:  # a new run (its own run dir) continuing from the crashed run's last checkpoint
        cmd += ["--resume", resume]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONPATH=str(REPO))
    t0 = time.time()
    with open(log, "w") as fh, open(log.with_suffix(".json"), "w") as js:
        rc = subprocess.call(cmd, stdout=js, stderr=fh, env=env, cwd=REPO)
    body = None
    text = log.with_suffix(".json").read_text()
    start = text.find("\n{")  # --json: the run summary (RCCL prints its banner to stdout first)
    try:
        body = json.loads(text[start + 1:] if start >= 0 else text) if text.strip() else None
    except json.JSONDecodeError:
        body = None
    print(f"[{run_id}{' resume' if resume else ''}] rc={rc} {time.time() - t0:.0f}s", file=sys.stderr, flush=True)
    return rc, body


def main() -> int:
    out = Path(sys.argv[1] if len(sys.argv) > 1 else REPO / "gpurun_out/xl_e2e").resolve()
    if out.exists():
        shutil.rmtree(out)
    out.mkdir(parents=True)
    shutil.rmtree(RUNS, ignore_errors=True)
    RUNS.mkdir(parents=True)
    free_gb = shutil.disk_usage(RUNS).free / 1e9
    if free_gb < 60:  # one run's two 18.7 GB checkpoints at once (the newer written before pruning)
        print(json.dumps({"status": "skipped", "reason": f"{free_gb:.0f} GB free"}))
        return 0
    a_cfg, b_cfg = _config(out, "xl-a", None), _config(out, "xl-b", 5)
    rc_a, res_a = _train(a_cfg, "xl-a", None, out / "a.log")
    shutil.rmtree(RUNS / "xl-a", ignore_errors=True)  # room for run B's checkpoints
    rc_b1, _ = _train(b_cfg, "xl-b", None, out / "b1.log")
    rc_b2, res_b = _train(b_cfg, "xl-b-resumed", "xl-b", out / "b2.log")
    shutil.rmtree(RUNS, ignore_errors=True)  # 18.7 GB checkpoints are not results
    summary = {"rc": [rc_a, rc_b1, rc_b2], "a": res_a, "b_resumed": res_b}
    ok = rc_a == 0 and rc_b1 != 0 and rc_b2 == 0 and res_a is not None and res_b is not None
    if ok:
        la = float(res_a["training"]["final_loss"])
        lb = float(res_b["training"]["final_loss"])
        summary.update(final_loss_a=la, final_loss_b=lb, abs_diff=abs(la - lb), pass_=abs(la - lb) <= 1e-5)
    summary["status"] = "ok" if ok and summary.get("pass_") else "fail"
    print(json.dumps(summary, default=str))
    return 0 if summary["status"] == "ok" else 1


if __name__ == "__main__":
    sys.exit(main())
