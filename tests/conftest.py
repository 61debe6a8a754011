"""Shared test configuration.

Markers: ``gpu`` (needs a MI355X; the driver runs ``-m gpu`` on a real box and ``-m "not gpu"``
here), ``slow`` (multi-process / long running).
"""

from __future__ import annotations

import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")


def pytest_configure(config: pytest.Config) -> None:
    config.addinivalue_line("markers", "gpu: requires an AMD Instinct MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")


def minimal_payload(**overrides: object) -> dict[str, object]:
    payload: dict[str, object] = {
        "schema_version": 1,
        "run": {"name": "test-run"},
        "model": {"name": "dummy_gpt"},
        "data": {"name": "dummy_text"},
        "trainer": {"max_steps": 5, "warmup_steps": 0, "micro_batch_size": 1, "grad_accum_steps": 1},
        "ddp": {},
        "mlflow": {"enabled": False},
        "logging": {"log_to_file": False},
        "output": {"root_dir": "runs"},
    }
    payload.update(overrides)
    return payload


_POLICY_ENV = ("LLMTRAIN_DET_SCHEDULE", "LLMTRAIN_WGRAD_STREAM")


@pytest.fixture(autouse=True)
def _isolated_kernel_policy():
    """Every test starts and ends with the same process-wide kernel policy (``ops._POLICY``, the
    C++ deterministic flag and the environment knobs that feed them): a test that switches
    deterministic mode, directly or through a Trainer, cannot change the routing of a later test —
    in particular the bench-shape step test always runs the routing it names."""
    from llmtrain import ops

    state = ops.policy_state()
    env = {k: os.environ.get(k) for k in _POLICY_ENV}
    yield
    ops.restore_policy(state)
    for k, v in env.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


@pytest.fixture
def in_tmp(tmp_path: Path, monkeypatch: pytest.MonkeyPatch) -> Path:
    monkeypatch.chdir(tmp_path)
    return tmp_path


@pytest.fixture(scope="session")
def gpu_device():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    from llmtrain.ops import _ext

    _ext.require()  # a GPU box without the built extension is a failure, not a skip
    return torch.device("cuda", 0)


class _ListHandler:
    pass


@pytest.fixture
def trainer_records():
    """Records emitted by the trainer logger, independent of how the CLI configured handlers."""
    import logging

    records: list[logging.LogRecord] = []

    class Collect(logging.Handler):
        def emit(self, record: logging.LogRecord) -> None:
            records.append(record)

    logger = logging.getLogger("llmtrain.training.trainer")
    handler = Collect(level=logging.DEBUG)
    old_level = logger.level
    logger.addHandler(handler)
    logger.setLevel(logging.INFO)
    try:
        yield records
    finally:
        logger.removeHandler(handler)
        logger.setLevel(old_level)
