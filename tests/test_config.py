"""Config schema + loader (reference tests/test_config.py): defaults, validators, strictness,
plugin extras, widened MI355X literals, and every shipped preset validating unchanged."""

from __future__ import annotations

from pathlib import Path

import pytest
import yaml

from llmtrain.config.loader import ConfigLoadError, load_and_validate_config
from llmtrain.config.schemas import RunConfig

PRESETS = sorted((Path(__file__).resolve().parents[1] / "configs" / "presets").glob("*.yaml"))


def _minimal() -> dict[str, object]:
    return {
        "schema_version": 1,
        "run": {"name": "test-run"},
        "model": {"name": "tiny-model"},
        "data": {"name": "toy-data"},
        "trainer": {},
        "ddp": {},
        "mlflow": {},
        "logging": {},
        "output": {},
    }


def _write(tmp_path: Path, payload: object) -> Path:
    path = tmp_path / "config.yaml"
    path.write_text(yaml.safe_dump(payload, sort_keys=False), encoding="utf-8")
    return path


def test_defaults_materialize(tmp_path: Path) -> None:
    path = _write(tmp_path, _minimal())
    cfg, raw, resolved = load_and_validate_config(str(path))
    assert raw == str(path) and resolved == path.resolve()
    assert cfg.run.seed == 1337 and cfg.run.device == "cpu" and cfg.run.precision == "fp32"
    assert cfg.model.block_size == 256 and cfg.model.d_model == 384 and cfg.model.dropout == 0.1
    assert cfg.model.extra == {} and cfg.data.extra == {} and cfg.trainer.extra == {}
    assert cfg.data.cache_dir == ".cache/datasets"
    assert cfg.trainer.lr == 3e-4 and cfg.trainer.warmup_steps == 100
    assert cfg.ddp.backend == "gloo" and cfg.ddp.timeout_sec == 1800
    assert cfg.logging.json_output is True
    assert cfg.output.root_dir == "runs"


@pytest.mark.parametrize(
    "model,trainer",
    [
        ({"name": "m", "d_model": 384, "n_heads": 7}, {}),
        ({"name": "m", "d_model": 256, "d_ff": 128}, {}),
        ({"name": "m"}, {"max_steps": 10, "warmup_steps": 20}),
        ({"name": "m", "block_size": 4}, {}),
        ({"name": "m", "dropout": 1.0}, {}),
    ],
)
def test_cross_field_and_range_validation(tmp_path: Path, model, trainer) -> None:
    payload = _minimal()
    payload["model"] = model
    payload["trainer"] = trainer
    with pytest.raises(ConfigLoadError) as info:
        load_and_validate_config(str(_write(tmp_path, payload)))
    assert info.value.errors and info.value.details


def test_extra_fields_rejected(tmp_path: Path) -> None:
    payload = _minimal()
    payload["run"] = {"name": "x", "extra": "nope"}
    with pytest.raises(ConfigLoadError):
        load_and_validate_config(str(_write(tmp_path, payload)))


def test_missing_section_rejected(tmp_path: Path) -> None:
    payload = _minimal()
    del payload["ddp"]
    with pytest.raises(ConfigLoadError):
        load_and_validate_config(str(_write(tmp_path, payload)))


def test_plugin_extras_accepted(tmp_path: Path) -> None:
    payload = _minimal()
    payload["model"] = {"name": "m", "extra": {"adapter": "dummy"}}
    payload["data"] = {"name": "d", "extra": {"dataset": "synthetic"}}
    payload["trainer"] = {"extra": {"gradient_clip": 0.9}}
    cfg, _, _ = load_and_validate_config(str(_write(tmp_path, payload)))
    assert cfg.model.extra["adapter"] == "dummy"
    assert cfg.data.extra["dataset"] == "synthetic"
    assert cfg.trainer.extra["gradient_clip"] == 0.9


@pytest.mark.parametrize("device", ["cuda", "rocm", "cpu", "mps"])
@pytest.mark.parametrize("backend", ["gloo", "nccl", "rccl"])
def test_widened_literals(device: str, backend: str) -> None:
    payload = _minimal()
    payload["run"] = {"name": "r", "device": device, "precision": "bf16"}
    payload["ddp"] = {"backend": backend}
    cfg = RunConfig.model_validate(payload)
    assert cfg.run.device == device and cfg.ddp.backend == backend


def test_frozen() -> None:
    cfg = RunConfig.model_validate(_minimal())
    with pytest.raises(Exception):
        cfg.run.seed = 3  # type: ignore[misc]


def test_yaml_errors_and_non_mapping(tmp_path: Path) -> None:
    bad = tmp_path / "bad.yaml"
    bad.write_text("run: [unclosed", encoding="utf-8")
    with pytest.raises(ConfigLoadError, match="YAML parse error"):
        load_and_validate_config(str(bad))
    seq = tmp_path / "seq.yaml"
    seq.write_text("- 1\n- 2\n", encoding="utf-8")
    with pytest.raises(ConfigLoadError, match="mapping"):
        load_and_validate_config(str(seq))
    with pytest.raises(ConfigLoadError, match="unable to read"):
        load_and_validate_config(str(tmp_path / "missing.yaml"))
    with pytest.raises(ConfigLoadError):
        load_and_validate_config("  ")


@pytest.mark.parametrize("preset", PRESETS, ids=[p.stem for p in PRESETS])
def test_reference_presets_validate(preset: Path) -> None:
    cfg, _, _ = load_and_validate_config(str(preset))
    assert cfg.run.name


def test_mi355x_presets_present() -> None:
    names = {p.stem for p in PRESETS}
    assert {"gpt2_124m_mi355x", "gpt2_124m_mi355x_ddp8", "gpt2_xl_mi355x_ddp8"} <= names
