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


def test_deterministic_mode_routes_the_lm_head_to_the_fixed_order_gemm() -> None:
    """run.deterministic: the LM-head logits take the fixed-order fused GEMM at any size (row
    chunks); the other forward / dX GEMMs above the size cap stay on the library.  Routing only
    (meta tensors): the GPU tests check the numerics."""
    from llmtrain import ops

    h = torch.empty(131072, 768, dtype=torch.bfloat16, device="meta")
    w = torch.empty(50304, 768, dtype=torch.bfloat16, device="meta")
    with ops.kernel_policy(False):
        assert not ops._fgemm_ok(h, 768, 50304, w, op="head")  # above the size cap: hipBLASLt
    with ops.kernel_policy(True, "serial"):
        assert ops._fgemm_ok(h, 768, 50304, w, op="head")
        assert not ops._fgemm_ok(h, 768, 2304, w, op="fwd")
        assert not ops._fgemm_ok(h, 768, 2304, w, op="dx")
