"""YAML → :class:`RunConfig` loading.

Behavioural parity with reference ``src/llmtrain/config/loader.py:14-65``: every failure mode
(empty path, unreadable file, YAML syntax error, non-mapping document, schema violation)
surfaces as one exception type, :class:`ConfigLoadError`, which the CLI maps to exit code 2.
"""

from __future__ import annotations

from pathlib import Path
from typing import Any

import yaml
from pydantic import ValidationError

from llmtrain.config.schemas import RunConfig

__all__ = ["ConfigLoadError", "load_and_validate_config", "load_yaml_config", "resolve_config_path"]


class ConfigLoadError(Exception):
    """A config could not be turned into a :class:`RunConfig`.

    ``message`` is a one-line description, ``details`` the verbose validator text (if any) and
    ``errors`` the structured Pydantic error list (empty for non-validation failures).
    """

    def __init__(self, message: str, details: str | None = None, errors: list[Any] | None = None):
        super().__init__(message)
        self.message = message
        self.details = details
        self.errors = list(errors) if errors else []


def resolve_config_path(config_path: str) -> tuple[str, Path]:
    """Return ``(as_given, absolute_resolved_path)``; relative paths resolve against the CWD."""
    if not isinstance(config_path, str) or not config_path.strip():
        raise ConfigLoadError("config path must be a non-empty string")
    candidate = Path(config_path).expanduser()
    if not candidate.is_absolute():
        candidate = Path.cwd() / candidate
    return config_path, candidate.resolve()


def load_yaml_config(config_path: Path) -> Any:
    """Parse a YAML file with the safe loader; an empty document becomes ``{}``."""
    try:
        text = config_path.read_text(encoding="utf-8")
    except OSError as exc:
        raise ConfigLoadError(f"unable to read config file {config_path}: {exc}") from exc
    try:
        document = yaml.safe_load(text)
    except yaml.YAMLError as exc:
        raise ConfigLoadError(f"YAML parse error in {config_path}: {exc}") from exc
    return {} if document is None else document


def load_and_validate_config(config_path: str) -> tuple[RunConfig, str, Path]:
    """Load + validate; returns ``(config, raw_path, resolved_path)``."""
    raw, resolved = resolve_config_path(config_path)
    document = load_yaml_config(resolved)
    if not isinstance(document, dict):
        raise ConfigLoadError(f"top-level config must be a mapping: {resolved}")
    try:
        config = RunConfig.model_validate(document)
    except ValidationError as exc:
        raise ConfigLoadError(
            f"validation failed for {resolved}", details=str(exc), errors=exc.errors()
        ) from exc
    return config, raw, resolved
