"""Shipped TunableOp GEMM table (llmtrain.runtime.tuning): well-formed, gfx950, CPU no-op."""

from __future__ import annotations

import torch

from llmtrain.runtime.tuning import TUNED_TABLE, enable_tuned_gemms


def test_table_is_well_formed_for_gfx950() -> None:
    rows = [line.split(",") for line in TUNED_TABLE.read_text().splitlines() if line.strip()]
    validators = {r[1]: r[2] for r in rows if r[0] == "Validator"}
    assert validators["GCN_ARCH_NAME"].startswith("gfx950")
    assert {"PT_VERSION", "HIPBLASLT_VERSION", "ROCBLAS_VERSION"} <= set(validators)
    entries = [r for r in rows if r[0] != "Validator"]
    assert entries and all(len(r) == 4 and float(r[3]) > 0 for r in entries)
    # the bench's LM-head GEMMs (vocab padded to 50304) are covered
    assert any("50304" in r[1] for r in entries)


def test_cpu_device_is_a_no_op() -> None:
    assert enable_tuned_gemms(torch.device("cpu")) is False
