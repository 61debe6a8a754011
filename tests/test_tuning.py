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


def test_tuned_bias_gemm_shapes_route_to_the_library(monkeypatch) -> None:
    """Bias-GEMM shapes with a measured library solution in the table (micro-batch 32 qkv / out
    forward) are routed away from the fused GEMM; other shapes and an unloaded table are not."""
    import llmtrain.ops as ops
    from llmtrain.runtime import tuning

    monkeypatch.setattr(ops, "_TUNED_BIAS_GEMMS", None)
    assert ops._library_tuned_bias_gemm(32768, 2304, 768) is False  # table not loaded here
    monkeypatch.setitem(tuning._state, "active", True)
    assert ops._library_tuned_bias_gemm(32768, 2304, 768)  # qkv forward, micro-batch 32
    assert ops._library_tuned_bias_gemm(32768, 768, 768)  # out-projection forward
    assert ops._library_tuned_bias_gemm(131072, 3072, 768)  # fc forward, micro-batch 128
    assert not ops._library_tuned_bias_gemm(32768, 3072, 768)  # fc forward at 32: fused GELU epilogue
    assert not ops._library_tuned_bias_gemm(4096, 2304, 768)

