"""Load → run directory → persisted config + meta (reference tests/test_integration_flow.py)."""

from __future__ import annotations

import json
from pathlib import Path

import pytest
import yaml

from llmtrain.config.loader import load_and_validate_config
from llmtrain.utils.metadata import generate_meta, write_meta_json
from llmtrain.utils.run_dir import create_run_directory, write_resolved_config

from conftest import minimal_payload


def test_run_directory_flow(tmp_path: Path) -> None:
    cfg_path = tmp_path / "c.yaml"
    cfg_path.write_text(yaml.safe_dump(minimal_payload()), encoding="utf-8")
    cfg, raw, resolved = load_and_validate_config(str(cfg_path))
    run_dir = create_run_directory(tmp_path / "runs", "rid")
    assert (run_dir / "logs").is_dir()
    write_resolved_config(run_dir, cfg)
    meta = generate_meta(run_id="rid", run_name=cfg.run.name, config_path=raw, resolved_config_path=str(resolved))
    write_meta_json(run_dir, meta)
    saved = yaml.safe_load((run_dir / "config.yaml").read_text())
    assert saved == cfg.model_dump()
    assert list(saved) == list(cfg.model_dump())  # schema order preserved
    m = json.loads((run_dir / "meta.json").read_text())
    assert m["meta_version"] == 1 and m["run_id"] == "rid" and m["created_at"].endswith("Z")
    assert set(m["ddp_env"]) == {"RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"}
    assert not list(run_dir.glob("*.tmp"))
    with pytest.raises(FileExistsError):
        create_run_directory(tmp_path / "runs", "rid")
