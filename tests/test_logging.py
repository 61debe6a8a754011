"""Structured logging (reference tests/test_logging.py)."""

from __future__ import annotations

import io
import json
import logging
from pathlib import Path

from llmtrain.utils.logging import configure_logging


def test_json_records_have_contract_keys() -> None:
    stream = io.StringIO()
    logger = configure_logging(name="llmtrain.test_json", stream=stream, json_output=True)
    logger.info("hello %s", "world")
    record = json.loads(stream.getvalue().strip().splitlines()[-1])
    assert set(record) == {"timestamp", "level", "logger", "message"}
    assert record["message"] == "hello world" and record["level"] == "INFO"


def test_idempotent_handlers_and_file(tmp_path: Path) -> None:
    stream = io.StringIO()
    log_file = tmp_path / "logs" / "train.log"
    for _ in range(3):
        logger = configure_logging(
            name="llmtrain.test_idem", stream=stream, log_to_file=True, file_name=str(log_file), json_output=False
        )
    assert len(logger.handlers) == 2 and logger.propagate is False
    logger.warning("to file")
    for h in logger.handlers:
        h.flush()
    assert "to file" in log_file.read_text()
    logger = configure_logging(name="llmtrain.test_idem", stream=stream, log_to_file=False)
    assert not any(isinstance(h, logging.FileHandler) for h in logger.handlers)
