"""Forward GEMM: ping-pong kernel (csrc/gemm_pp.hip) vs hipBLASLt (torch.addmm) vs gemm_fused.

    python bench/gemm_pp.py check           # numerics vs fp32 (shapes, ragged M / N, bias, GELU)
    python bench/gemm_pp.py time [--tokens M] [--only pp,blas,fused]   # forward and dX shapes

Each timing line: kernel, shape, ms (median of 20), TFLOP/s on the 2*M*N*K GEMM FLOPs.
LLMT_GPP_FILL=3 selects the fills-inside-MFMA schedule (default 1: fills in the LOAD segment).
"""

from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parent))
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from micro import timeit  # noqa: E402

SHAPES = {"qkv": (2304, 768), "out": (768, 768), "fc": (3072, 768), "proj": (768, 3072)}  # (N, K)
# data gradients dX = dY W, W = nn.Linear weight [out, in]: (N = in, K = out); proj's carries the GELU backward
DX_SHAPES = {"qkv_dx": (768, 2304), "out_dx": (768, 768), "fc_dx": (768, 3072), "proj_dx_gelu": (3072, 768)}


def _ops():
    from llmtrain.ops import _ext

    _ext.require()
    return torch.ops.llmtrain_hip


def check() -> int:
    ops = _ops()
    torch.manual_seed(0)
    bad = 0
    cases = [(4096, n, k, name) for name, (n, k) in SHAPES.items()]
    cases += [(1000, 2304, 768, "ragged M"), (300, 776, 128, "ragged N, K 128"), (64, 50304, 768, "head rows")]
    for M, N, K, name in cases:
        for epi in (0, 1):
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            w = (torch.randn(N, K, device="cuda") * K**-0.5).to(torch.bfloat16)
            b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
            out, out2 = ops.gemm_pp(x, w, b, epi)
            ref = (x.float() @ w.float().t() + b.float())
            err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
            ok = err < 1e-2
            row = {"case": name, "M": M, "N": N, "K": K, "epi": epi, "rel_err": err}
            if epi == 1:
                gref = F.gelu(out.float())
                gerr = ((out2.float() - gref).abs().max() / gref.abs().max()).item()
                row["gelu_rel_err"] = gerr
                ok = ok and gerr < 1e-2
            row["ok"] = ok
            bad += not ok
            print(json.dumps(row), flush=True)
    dx_cases = [(4096, n, k, name) for name, (n, k) in DX_SHAPES.items()] + [(1000, 776, 128, "dx ragged")]
    for M, N, K, name in dx_cases:
        for epi in (0, 2):
            dy = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            w = (torch.randn(K, N, device="cuda") * K**-0.5).to(torch.bfloat16)  # [K_red, N]
            u = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
            out, _ = ops.gemm_pp(dy, w, None, epi, True, u if epi == 2 else None)
            ref = dy.float() @ w.float()
            if epi == 2:
                x = u.float().requires_grad_(True)
                F.gelu(x).backward(torch.ones_like(x))
                ref = ref * x.grad
            err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
            ok = err < 1e-2
            bad += not ok
            print(json.dumps({"case": name, "M": M, "N": N, "K": K, "kn": True, "epi": epi, "rel_err": err, "ok": ok}),
                  flush=True)
    # out-projection dX + attention row constants (epilogue 3): dO = dy @ Wo, delta = per-head dO . O
    T = 1024
    for M in (4096, 2048):
        dy = torch.randn(M, 768, device="cuda", dtype=torch.bfloat16)
        w = (torch.randn(768, 768, device="cuda") * 768**-0.5).to(torch.bfloat16)
        o = torch.randn(M, 768, device="cuda", dtype=torch.bfloat16)
        d_o, delta = ops.gemm_pp(dy, w, None, 3, True, o, T)
        ref = dy.float() @ w.float()
        err = ((d_o.float() - ref).abs().max() / ref.abs().max()).item()
        dref = (d_o.float() * o.float()).view(M // T, T, 12, 64).sum(-1).permute(0, 2, 1)
        derr = ((delta - dref).abs().max() / dref.abs().max()).item()
        ok = err < 1e-2 and derr < 1e-4
        bad += not ok
        print(json.dumps({"case": "dx_attn delta", "M": M, "rel_err": err, "delta_rel_err": derr, "ok": ok}), flush=True)
    return 1 if bad else 0


def time_shapes(M: int, only: str = "") -> None:
    ops = _ops()
    for name, (N, K) in SHAPES.items():
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") * K**-0.5).to(torch.bfloat16)
        b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
        flops = 2.0 * M * N * K
        variants = {
            "pp": lambda: ops.gemm_pp(x, w, b, 0),
            "pp_gelu": lambda: ops.gemm_pp(x, w, b, 1),
            "blas": lambda: torch.addmm(b, x, w.t()),
            "fused": lambda: ops.gemm_fused(x[:16384], w, False, 0, b),
        }
        for label, fn in variants.items():
            if only and label not in only.split(","):
                continue
            if label == "pp_gelu" and name != "fc":
                continue
            ms = timeit(fn)
            f = flops * (16384 / M if label == "fused" else 1.0)
            print(json.dumps({"M": M, "gemm": name, "variant": label, "ms": round(ms, 4),
                              "TFLOPs": round(f / ms / 1e9, 1)}), flush=True)


def time_dx(M: int, only: str = "") -> None:
    ops = _ops()
    for name, (N, K) in DX_SHAPES.items():
        dy = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = (torch.randn(K, N, device="cuda") * K**-0.5).to(torch.bfloat16)
        u = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        gelu = name.endswith("gelu")
        flops = 2.0 * M * N * K
        attn = name == "out_dx"
        variants = {
            "pp": lambda: ops.gemm_pp(dy, w, None, 2 if gelu else (3 if attn else 0), True,
                                      u if (gelu or attn) else None, 1024 if attn else 0),
            "blas": lambda: torch.mm(dy, w),
            "fused": lambda: ops.gemm_fused(dy[:16384], w, True, 2 if gelu else (3 if attn else 0), None,
                                            u[:16384] if (gelu or attn) else None, None, 1024 if attn else 0),
        }
        for label, fn in variants.items():
            if only and label not in only.split(","):
                continue
            ms = timeit(fn)
            f = flops * (16384 / M if label == "fused" else 1.0)
            print(json.dumps({"M": M, "gemm": name, "variant": label, "ms": round(ms, 4),
                              "TFLOPs": round(f / ms / 1e9, 1)}), flush=True)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["check", "time"])
    ap.add_argument("--only", default="", help="comma-separated variant labels (time)")
    ap.add_argument("--tokens", type=int, default=131072)
    args = ap.parse_args()
    if args.what == "check":
        return check()
    time_shapes(args.tokens, args.only)
    time_dx(args.tokens, args.only)
    return 0


if __name__ == "__main__":
    sys.exit(main())
