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
