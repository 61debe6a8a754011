"""The environment knobs the tree reads — the complete list (``scripts/lint.py`` fails on a
``LLMTRAIN_*`` / ``LLMT_*`` variable read anywhere in ``llmtrain/``, ``csrc/`` or ``bench.py``
that is not listed here, on more than 12 of them, and on a ``docs/debugging.md`` knob table that
differs from this one).  Kernel schedule variants that lost their A/B were deleted with their
knobs (git history and ``docs/round*.md`` record what they measured); none are read from C++.
"""

from __future__ import annotations

__all__ = ["KNOBS", "MAX_KNOBS"]

MAX_KNOBS = 12

# name -> (default, effect)
KNOBS: dict[str, tuple[str, str]] = {
    "LLMTRAIN_DET_SCHEDULE": (
        "serial",
        "`run.deterministic` GEMM schedule: `serial` (one stream, tuned hipBLASLt forward / dX, "
        "LM-head dX on the fixed-order kernel) or `ours` (every forward / dX GEMM on csrc/gemm_fused.hip)",
    ),
    "LLMTRAIN_WGRAD_STREAM": (
        "0",
        "1: weight-gradient GEMMs on a side stream beside the main stream (one stream measured faster "
        "since round 4, profiles/r4/ab_side_stream_vs_one_stream_mb*.txt)",
    ),
    "LLMTRAIN_FUSED_GEMM": (
        "1",
        "0: plain hipBLASLt GEMMs with separate GELU / attention-delta passes instead of the fused-epilogue "
        "GEMM ops",
    ),
    "LLMTRAIN_FGEMM_MAX_A_MB": ("64", "fused-GEMM routing: operand size (MiB) above which a GEMM stays on hipBLASLt"),
    "LLMTRAIN_FGEMM_ANY": ("dx_gelu,dx_attn", "fused-GEMM ops taken at any operand size"),
    "LLMTRAIN_FGEMM_NEVER": ("(none)", "fused-GEMM ops that always stay on hipBLASLt"),
    "LLMTRAIN_TUNED_GEMMS": ("1", "0: do not load the shipped hipBLASLt TunableOp table (llmtrain/runtime/tuning.py)"),
    "LLMTRAIN_ROCTX": ("0", "1: roctx ranges per engine phase / block (rocprofv3 --marker-trace)"),
    "LLMTRAIN_DEBUG_KERNELS": ("0", "1: load `_llmtrain_hip_debug.so` (device-side bounds asserts) instead of the release build"),
    "LLMTRAIN_HIP_EXT": ("in-tree .so", "path of the HIP extension to load (A/B of two builds in one tree)"),
}
