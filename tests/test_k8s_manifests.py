"""Static checks of the Kubernetes assets (the reference tests them only with a live kind
cluster, k8s/test_e2e.sh): every manifest parses, embedded training configs validate against
the schema, each IndexedJob's WORLD_SIZE equals its completions, and the shell scripts parse."""

from __future__ import annotations

import subprocess
from pathlib import Path

import pytest
import yaml

from llmtrain.config.schemas import RunConfig

ROOT = Path(__file__).resolve().parents[1]
MANIFESTS = sorted((ROOT / "k8s").rglob("*.yaml"))


@pytest.mark.parametrize("path", MANIFESTS, ids=lambda p: str(p.relative_to(ROOT)))
def test_manifest_parses(path: Path) -> None:
    docs = [d for d in yaml.safe_load_all(path.read_text()) if d is not None]
    assert docs, path
    for doc in docs:
        assert "kind" in doc and "apiVersion" in doc


def _docs(kind: str) -> list[tuple[Path, dict]]:
    out = []
    for path in MANIFESTS:
        for doc in yaml.safe_load_all(path.read_text()):
            if doc and doc.get("kind") == kind:
                out.append((path, doc))
    return out


def test_embedded_train_configs_validate() -> None:
    maps = _docs("ConfigMap")
    assert len(maps) >= 2
    for _, doc in maps:
        cfg = RunConfig.model_validate(yaml.safe_load(doc["data"]["train.yaml"]))
        assert cfg.ddp.enabled


def test_jobs_world_size_matches_completions() -> None:
    jobs = [(p, j) for p, j in _docs("Job") if j["spec"].get("completionMode") == "Indexed"]
    assert len(jobs) >= 2
    for path, job in jobs:
        spec = job["spec"]
        env = {e["name"]: e.get("value") for e in spec["template"]["spec"]["containers"][0]["env"]}
        assert int(env["WORLD_SIZE"]) == spec["completions"] == spec["parallelism"], path
        gpu = spec["template"]["spec"]["containers"][0].get("resources", {}).get("limits", {}).get("amd.com/gpu")
        if gpu is not None:
            assert gpu == 1  # one MI355X per pod, one rank per GPU


@pytest.mark.parametrize("script", ["k8s/entrypoint.sh", "k8s/test_e2e.sh"])
def test_shell_scripts_parse(script: str) -> None:
    subprocess.run(["bash", "-n", str(ROOT / script)], check=True)


@pytest.mark.parametrize("script", ["k8s/gang_restart.sh"])
def test_more_scripts_parse(script: str) -> None:
    subprocess.run(["bash", "-n", str(ROOT / script)], check=True)


def test_jobs_fail_as_a_gang() -> None:
    """Any rank failure fails the whole Job (a replaced pod cannot rejoin a live RCCL group): no
    per-index retries, FailJob on every non-zero exit and on disruption."""
    for path, job in _docs("Job"):
        spec = job["spec"]
        assert spec.get("backoffLimit") == 0 and "backoffLimitPerIndex" not in spec, path
        rules = spec["podFailurePolicy"]["rules"]
        exit_rule = next(r for r in rules if "onExitCodes" in r)
        assert exit_rule["action"] == "FailJob"
        assert exit_rule["onExitCodes"]["operator"] == "NotIn" and exit_rule["onExitCodes"]["values"] == [0]
        assert any(r["action"] == "FailJob" and r.get("onPodConditions") for r in rules)


FAKE_KUBECTL = r"""#!/usr/bin/env bash
# kubectl stand-in: each `apply` starts a new Job attempt; attempts < $FAIL_ATTEMPTS end Failed
state="$STATE_DIR/attempts"
[ -f "$state" ] || echo 0 > "$state"
case "$1" in
  apply) echo $(( $(cat "$state") + 1 )) > "$state"; echo "job.batch/llmtrain created" ;;
  delete) ;;
  get)
    if [ "$2" = job ]; then
      if [ "$(cat "$state")" -le "$FAIL_ATTEMPTS" ]; then echo -n "FailureTarget Failed "; else echo -n "Complete "; fi
    else
      printf 'llmtrain-1-abc 1 Error\nllmtrain-0-def 0 Completed\n'
    fi ;;
esac
"""


def _run_controller(tmp_path: Path, fail_attempts: int, max_restarts: int) -> subprocess.CompletedProcess:
    import os

    fake = tmp_path / "kubectl"
    fake.write_text(FAKE_KUBECTL)
    fake.chmod(0o755)
    env = dict(os.environ, KUBECTL=str(fake), STATE_DIR=str(tmp_path), FAIL_ATTEMPTS=str(fail_attempts))
    return subprocess.run(
        ["bash", str(ROOT / "k8s" / "gang_restart.sh"), "--max-restarts", str(max_restarts), "--poll", "0",
         "--timeout", "60"], env=env, capture_output=True, text=True, timeout=120,
    )


def test_gang_restart_recovers_after_a_failed_attempt(tmp_path: Path) -> None:
    proc = _run_controller(tmp_path, fail_attempts=1, max_restarts=2)
    assert proc.returncode == 0, proc.stdout + proc.stderr
    assert "attempt 0: job/llmtrain failed" in proc.stdout
    assert "failed pod llmtrain-1-abc exit=1 reason=Error" in proc.stdout
    assert "complete after 1 restart(s)" in proc.stdout
    assert (tmp_path / "attempts").read_text().strip() == "2"


def test_gang_restart_gives_up(tmp_path: Path) -> None:
    proc = _run_controller(tmp_path, fail_attempts=99, max_restarts=2)
    assert proc.returncode == 1
    assert "giving up after 2 restart(s)" in proc.stdout
    assert (tmp_path / "attempts").read_text().strip() == "3"


def _env(job: dict) -> dict:
    return {e["name"]: e for e in job["spec"]["template"]["spec"]["containers"][0]["env"]}


def test_single_pod_fallback_job() -> None:
    """k8s/job-1pod8gpu.yaml: one pod, all 8 GPUs, torchrun inside (docs/k8s.md fallback)."""
    job = yaml.safe_load((ROOT / "k8s" / "job-1pod8gpu.yaml").read_text())
    spec = job["spec"]
    assert spec["completions"] == spec["parallelism"] == 1
    c = spec["template"]["spec"]["containers"][0]
    assert c["resources"]["limits"]["amd.com/gpu"] == 8
    env = _env(job)
    assert env["LAUNCH_MODE"]["value"] == "torchrun" and env["NPROC"]["value"] == "8"
    vols = {v["name"] for v in spec["template"]["spec"]["volumes"]}
    assert {"config", "runs", "mlflow", "dshm"} <= vols


def test_jobs_share_restart_identity_and_leave_nccl_debug_to_the_trainer() -> None:
    for path, job in _docs("Job"):
        env = _env(job)
        field = env["JOB_UID"]["valueFrom"]["fieldRef"]["fieldPath"]
        assert "controller-uid" in field, path  # one value per Job incarnation, shared by its pods
        assert "NCCL_DEBUG" not in env, path  # llmtrain.parallel.comm captures the transport lines


def _launch(*args: str, env: dict | None = None) -> subprocess.CompletedProcess:
    import os
    import sys

    full = dict(os.environ, PYTHONPATH=str(ROOT), **(env or {}))
    return subprocess.run([sys.executable, "-m", "llmtrain.launch", *args], env=full, capture_output=True,
                          text=True, timeout=120)


def test_latest_checkpoint_across_restarts(tmp_path: Path) -> None:
    from llmtrain.launch import latest_checkpoint

    assert latest_checkpoint(tmp_path, "job") is None
    for run, steps in {"job": [2, 4], "job-restart-ab12": [6, 10], "jobx": [99], "other": [50]}.items():
        d = tmp_path / run / "checkpoints"
        d.mkdir(parents=True)
        for s in steps:
            (d / f"step_{s:06d}.pt").write_bytes(b"x")
    (tmp_path / "job" / "checkpoints" / "step_000012.pt.tmp").write_bytes(b"partial")  # never picked
    assert latest_checkpoint(tmp_path, "job") == tmp_path / "job-restart-ab12" / "checkpoints" / "step_000010.pt"
    proc = _launch("latest-checkpoint", "--runs-root", str(tmp_path), "--run-id", "job")
    assert proc.returncode == 0 and proc.stdout.strip().endswith("job-restart-ab12/checkpoints/step_000010.pt")
    assert _launch("latest-checkpoint", "--runs-root", str(tmp_path), "--run-id", "none").returncode == 1


def test_restart_tag_is_shared_by_the_gang() -> None:
    from llmtrain.launch import restart_tag

    uid = "3F2A9C1E-77aa-4b1c-9d0e-123456789abc"
    assert restart_tag({"JOB_UID": uid}) == restart_tag({"JOB_UID": uid}) == "3f2a9c1e77aa"
    with pytest.raises(RuntimeError):
        restart_tag({})
    assert _launch("restart-tag", env={"JOB_UID": uid}).stdout.strip() == "3f2a9c1e77aa"
