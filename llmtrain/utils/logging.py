"""Structured logging for the ``llmtrain`` logger tree.

Reference behaviour (``utils/logging.py:11-90``): one-line JSON records
``{timestamp, level, logger, message[, exc_info]}`` (or a plain text format), an idempotent
stream handler (stdout unless a stream is given), an optional file handler that replaces any
previous one, and ``propagate=False`` on the configured logger.
"""

from __future__ import annotations

import json
import logging
import sys
from datetime import datetime, timezone
from pathlib import Path
from typing import Any, TextIO

__all__ = ["JsonFormatter", "configure_logging"]

_TEXT_FORMAT = "%(asctime)s %(levelname)s %(name)s: %(message)s"


class JsonFormatter(logging.Formatter):
    """One JSON object per line."""

    def format(self, record: logging.LogRecord) -> str:  # noqa: A003
        payload: dict[str, Any] = {
            "timestamp": datetime.fromtimestamp(record.created, tz=timezone.utc).isoformat(),
            "level": record.levelname,
            "logger": record.name,
            "message": record.getMessage(),
        }
        if record.exc_info:
            payload["exc_info"] = self.formatException(record.exc_info)
        return json.dumps(payload, ensure_ascii=True)


def _formatter(json_output: bool) -> logging.Formatter:
    return JsonFormatter() if json_output else logging.Formatter(_TEXT_FORMAT)


def _drop_file_handlers(logger: logging.Logger, keep: Path | None = None) -> logging.FileHandler | None:
    kept = None
    for handler in list(logger.handlers):
        if not isinstance(handler, logging.FileHandler):
            continue
        if keep is not None and Path(handler.baseFilename) == keep.resolve():
            kept = handler
            continue
        logger.removeHandler(handler)
        handler.close()
    return kept


def configure_logging(
    *,
    level: int = logging.INFO,
    name: str = "llmtrain",
    json_output: bool = True,
    log_to_file: bool = False,
    file_name: str = "train.log",
    stream: TextIO | None = None,
) -> logging.Logger:
    logger = logging.getLogger(name)
    logger.setLevel(level)
    fmt = _formatter(json_output)
    target = sys.stdout if stream is None else stream

    stream_handler = None
    for handler in logger.handlers:
        if (
            isinstance(handler, logging.StreamHandler)
            and not isinstance(handler, logging.FileHandler)
            and getattr(handler, "stream", None) is target
        ):
            stream_handler = handler
            break
    if stream_handler is None:
        stream_handler = logging.StreamHandler(target)
        logger.addHandler(stream_handler)
    stream_handler.setFormatter(fmt)

    if log_to_file:
        path = Path(file_name)
        path.parent.mkdir(parents=True, exist_ok=True)
        file_handler = _drop_file_handlers(logger, keep=path)
        if file_handler is None:
            file_handler = logging.FileHandler(path, encoding="utf-8")
            logger.addHandler(file_handler)
        file_handler.setFormatter(fmt)
    else:
        _drop_file_handlers(logger)

    logger.propagate = False
    return logger
