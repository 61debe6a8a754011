"""Bitwise repeatability of the hand-written kernels at production shapes (deterministic mode).

    python bench/repeat_check.py [M] [reps]

Each op runs ``reps`` times on identical inputs; every output is compared bitwise with the first
run.  A mismatch in a kernel with fixed-order reductions means a race (e.g. LDS reuse or a missing
wait), which the tolerance-based numerics tests would not see.  One JSON line per op.
"""

from __future__ import annotations

import json
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def _with(acc, fn):
    """Run ``fn(acc)`` and return its output together with the accumulator(s) it wrote."""
    return fn(acc), acc


def main() -> None:
    from llmtrain import ops
    from llmtrain.ops import _ext

    _ext.require()
    ops.set_deterministic(True)
    hip = torch.ops.llmtrain_hip
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    d, T, H = 768, 1024, 12
    B = M // T
    g = torch.Generator(device="cuda").manual_seed(0)
    bf = dict(device="cuda", dtype=torch.bfloat16)

    def rnd(*shape, scale=1.0, dtype=torch.bfloat16):
        return (torch.randn(*shape, device="cuda", generator=g) * scale).to(dtype)

    x768, x3072, x2304 = rnd(M, d), rnd(M, 4 * d), rnd(M, 3 * d)
    w_qkv, w_fc = rnd(3 * d, d, scale=0.02), rnd(4 * d, d, scale=0.02)
    w_proj, w_out = rnd(d, 4 * d, scale=0.02), rnd(d, d, scale=0.02)
    bias3 = torch.randn(3 * d, device="cuda", generator=g).to(**bf)
    bias4 = torch.randn(4 * d, device="cuda", generator=g).to(**bf)
    u = rnd(M, 4 * d)
    qkv = rnd(M, 3 * d)
    out, lse = hip.attn_fwd(qkv, B, T, H, 0.0, 0, None)
    dout = rnd(M, d)
    xs = torch.randn(M, d, device="cuda", generator=g)
    w_ln = torch.ones(d, device="cuda")
    _, _, mu, rs = hip.add_layernorm_fwd(xs, None, w_ln, torch.zeros(d, device="cuda"), 1e-5, torch.bfloat16)
    dres = torch.randn(M, d, device="cuda", generator=g)

    def f32z(n):
        return torch.zeros(n, device="cuda")

    from llmtrain.runtime.tuning import enable_tuned_gemms

    enable_tuned_gemms(torch.device("cuda"))  # the library GEMMs exactly as the trainer issues them
    lib_cases = {
        "hipblaslt fwd proj (addmm)": lambda: torch.addmm(bias3[:d], x3072, w_proj.t()),
        "hipblaslt dx fc (mm)": lambda: torch.mm(x3072, w_fc),
        "hipblaslt dx qkv (mm)": lambda: torch.mm(x2304, w_qkv),
        "hipblaslt fwd qkv (addmm)": lambda: torch.addmm(bias3, x768, w_qkv.t()),
    }
    cases = {
        "fgemm fwd qkv (bias)": lambda: hip.gemm_fused(x768, w_qkv, False, 0, bias3),
        "fgemm fwd fc (bias+gelu)": lambda: hip.gemm_fused(x768, w_fc, False, 1, bias4),
        "fgemm fwd proj": lambda: hip.gemm_fused(x3072, w_proj, False, 0, None),
        "fgemm dx qkv": lambda: hip.gemm_fused(x2304, w_qkv, True, 0),
        "fgemm dx fc": lambda: hip.gemm_fused(x3072, w_fc, True, 0),
        "fgemm dx proj+dgelu": lambda: _with(f32z(4 * d), lambda db: hip.gemm_fused(x768, w_proj, True, 2, None, u, db)[0]),
        "fgemm dx out+delta": lambda: hip.gemm_fused(dout, w_out, True, 3, None, out, f32z(d), T),
        "attn fwd": lambda: hip.attn_fwd(qkv, B, T, H, 0.0, 0, None),
        "attn bwd": lambda: _with(
            f32z(3 * d), lambda db: hip.attn_bwd(dout, qkv, out, lse, B, T, H, 0.0, 0, db, None, None)
        ),
        "ln bwd": lambda: _with(
            (f32z(d), f32z(d), f32z(d)), lambda a: hip.layernorm_bwd(dout, xs, mu, rs, w_ln, dres, a[0], a[1], None, True, a[2])
        ),
        "wgrad fc (det slabs)": lambda: _with(
            torch.zeros(4 * d, d, device="cuda"), lambda c: hip.wgrad_gemm_pp(u, x768, c, None, 0, -1)
        ),
        "wgrad qkv (det slabs)": lambda: _with(
            torch.zeros(3 * d, d, device="cuda"), lambda c: hip.wgrad_gemm_pp(x2304, x768, c, None, 0, -1)
        ),
    }

    def flat(o):
        if isinstance(o, torch.Tensor):
            return [o.detach().clone()]
        if isinstance(o, (tuple, list)):
            return [t for x in o for t in flat(x)]
        return []

    # NOISE=1: every repetition runs beside a stream of large GEMMs (the way the side stream's weight
    # gradients share the chip in a training step), so a timing-dependent race would show
    noise = os.environ.get("NOISE", "0") == "1"
    side = torch.cuda.Stream()
    na, nb = rnd(8192, 8192), rnd(8192, 8192)

    def run(fn):
        if noise:
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(6):
                    torch.mm(na, nb)
        out = fn()
        torch.cuda.synchronize()
        return out

    if os.environ.get("LIB", "0") == "1":
        cases = lib_cases
    for name, fn in cases.items():
        ref = flat(run(fn))
        bad = 0
        worst = 0.0
        for _ in range(reps - 1):
            got = flat(run(fn))
            for a, b in zip(ref, got):
                if not torch.equal(a, b):
                    bad += 1
                    diff = (a.float() - b.float()).abs()
                    worst = max(worst, float(diff.max()))
        print(json.dumps({"op": name, "M": M, "reps": reps, "noise": noise, "mismatching_outputs": bad,
                          "max_abs_diff": worst}), flush=True)


if __name__ == "__main__":
    main()
