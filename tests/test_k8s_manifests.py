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
    jobs = _docs("Job")
    assert len(jobs) >= 2
    for path, job in jobs:
        spec = job["spec"]
        assert spec["completionMode"] == "Indexed"
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
