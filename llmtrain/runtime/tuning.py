"""Shipped GEMM solution table for the library GEMMs (PyTorch TunableOp over hipBLASLt/rocBLAS).

The forward/dX GEMMs that stay on hipBLASLt (``torch.mm`` / ``addmm`` with the bias epilogue, and
the LM head) pick their kernel from the library heuristics.  ``scripts/tune_gemms.sh`` benchmarks
every hipBLASLt and rocBLAS solution for each (op, shape) the bench issues on an MI355X and writes
the winners to a CSV; that table ships in ``llmtrain/runtime/tuned/`` and is loaded here with
tuning OFF, so a run only looks solutions up (no benchmarking, no file writes).  Shapes not in the
table fall back to the heuristics.  TunableOp validates the table's PyTorch / HIP / hipBLASLt /
rocBLAS versions and GPU arch and ignores it on any mismatch.

``LLMTRAIN_TUNED_GEMMS=0`` disables it; a caller that set ``PYTORCH_TUNABLEOP_*`` itself keeps
full control (nothing is changed then).  Measured same-box A/B: +0.45 % bench (docs/performance.md).
"""

from __future__ import annotations

import logging
import os
from pathlib import Path

import torch

__all__ = ["TUNED_TABLE", "enable_tuned_gemms", "tuned_gemms_active"]

logger = logging.getLogger(__name__)

TUNED_TABLE = Path(__file__).with_name("tuned") / "gemm_tunableop_gfx950.csv"
_state: dict[str, bool] = {}


def enable_tuned_gemms(device: torch.device) -> bool:
    """Load the shipped table for ``device`` (idempotent).  Returns whether it is active."""
    if device.type != "cuda":
        return False
    if "active" in _state:
        return _state["active"]
    active = False
    if os.environ.get("LLMTRAIN_TUNED_GEMMS", "1") == "0":
        logger.info("tuned GEMM table disabled (LLMTRAIN_TUNED_GEMMS=0)")
    elif any(k.startswith("PYTORCH_TUNABLEOP_") for k in os.environ):
        logger.info("PYTORCH_TUNABLEOP_* set by the caller: leaving TunableOp as configured")
    elif not TUNED_TABLE.is_file():
        logger.info("no tuned GEMM table at %s", TUNED_TABLE)
    else:
        arch = torch.cuda.get_device_properties(device).gcnArchName
        if not arch.startswith("gfx950"):
            logger.info("tuned GEMM table is for gfx950, device is %s: not loaded", arch)
        else:
            tunable = torch.cuda.tunable
            tunable.tuning_enable(False)  # look-ups only: never benchmark, never write the file
            tunable.set_filename(str(TUNED_TABLE), insert_device_ordinal=False)
            tunable.enable(True)
            active = bool(tunable.read_file(str(TUNED_TABLE)))
            if not active:
                tunable.enable(False)
                logger.warning("tuned GEMM table %s rejected (version/arch validators); using heuristics", TUNED_TABLE)
            else:
                logger.info("tuned GEMM table loaded: %s", TUNED_TABLE)
    _state["active"] = active
    return active


def tuned_gemms_active() -> bool:
    """Whether :func:`enable_tuned_gemms` loaded the shipped table in this process."""
    return _state.get("active", False)
