"""Weight-gradient GEMM (csrc/gemm_wgrad_pp.hip): numerics and per-shape timing.

    python bench/wgrad_pp.py check            # numerics vs fp32 (every shape, bias, strided dy)
    python bench/wgrad_pp.py time [--tokens M] [--model gpt2-124m|gpt2-xl|head] [--only pp_slab,pp_slab_square]
    python bench/wgrad_pp.py sweep2 [--tokens M] [--model ...] [--splits 0,2] [--ssplits 0,4]  # tail tiling
    python bench/wgrad_pp.py sweep [--tokens M] [--model ...] [--splits 1,2,4] [--mode 0]
                                              # fixed split counts (the planner's choice as split 0)

Each timing line: kernel, shape, ms (median of 20), TFLOP/s on the 2*M*N*K GEMM FLOPs.
"""

from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from micro import timeit  # noqa: E402

SHAPES = {
    "gpt2-124m": {"qkv": (2304, 768), "out": (768, 768), "fc": (3072, 768), "proj": (768, 3072)},
    "gpt2-xl": {"qkv": (4800, 1600), "out": (1600, 1600), "fc": (6400, 1600), "proj": (1600, 6400)},
    "head": {"head": (50257, 768)},
}


def _ops():
    from llmtrain.ops import _ext

    _ext.require()
    return torch.ops.llmtrain_hip


def check() -> int:
    ops = _ops()
    torch.manual_seed(0)
    bad = 0
    cases = [(4096, n, k, name) for model in ("gpt2-124m", "gpt2-xl") for name, (n, k) in SHAPES[model].items()]
    cases += [(1000, 2304, 768, "ragged M"), (3 * 32 + 5, 768, 768, "tiny M"), (2048, 50257, 768, "head")]
    for M, N, K, name in cases:
        for mode in (-1, 0, 2):
            lda = 50304 if N == 50257 else N
            base = torch.randn(M, lda, device="cuda", dtype=torch.bfloat16)
            dy = base[:, :N]
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            c0 = torch.randn(N, K, device="cuda")
            b0 = torch.randn(N, device="cuda")
            c, b = c0.clone(), b0.clone()
            ops.wgrad_gemm_pp(dy, x, c, b, 0, mode)
            ref = c0 + dy.float().t() @ x.float()
            rb = b0 + dy.float().sum(0)
            err = ((c - ref).abs().max() / ref.abs().max()).item()
            berr = ((b - rb).abs().max() / rb.abs().max()).item()
            ok = err < 2e-5 and berr < 2e-5
            bad += not ok
            print(json.dumps({"case": name, "M": M, "N": N, "K": K, "mode": mode, "rel_err": err,
                              "bias_rel_err": berr, "ok": ok}), flush=True)
    # run-to-run bitwise (slab mode)
    dy = torch.randn(8192, 2304, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(8192, 768, device="cuda", dtype=torch.bfloat16)
    outs = []
    for _ in range(3):
        c = torch.zeros(2304, 768, device="cuda")
        ops.wgrad_gemm_pp(dy, x, c, None, 0, 0)
        outs.append(c)
    same = all(torch.equal(outs[0], o) for o in outs[1:])
    bad += not same
    print(json.dumps({"case": "slab mode bitwise repeat", "ok": same}), flush=True)
    return 1 if bad else 0


def _plan(ops, M, N, K, lda, bias, mode):
    keys = ("swap", "tiles", "split", "chunk", "mode", "nwg", "s_tiles", "s_split", "s_chunk", "s_mode", "s_nwg", "model_ns")
    return dict(zip(keys, ops.wgrad_pp_plan(M, N, K, lda, K, bias, 0, mode)))


def time_shapes(model: str, M: int, only: str = "", rounds: int = 1) -> None:
    """Time each shape's variants; with ``only`` the variants run in that order, ``rounds`` times
    (interleaved A/B)."""
    ops = _ops()
    _warm()
    for name, (N, K) in SHAPES[model].items():
        lda = 50304 if N == 50257 else N
        dy = torch.randn(M, lda, device="cuda", dtype=torch.bfloat16)[:, :N]
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        acc = torch.zeros(N, K, device="cuda")
        bias = torch.zeros(N, device="cuda")
        flops = 2.0 * M * N * K
        variants = {
            "pp_auto": lambda: ops.wgrad_gemm_pp(dy, x, acc, None, 0, -1),
            "pp_slab": lambda: ops.wgrad_gemm_pp(dy, x, acc, None, 0, 0),
            "pp_atomic": lambda: ops.wgrad_gemm_pp(dy, x, acc, None, 0, 2),
            "pp_slab_bias": lambda: ops.wgrad_gemm_pp(dy, x, acc, bias, 0, 0),
            # 256 x 256 tiles only (mode + 8): the rounds-1-5 tiling, A/B of the d = 1600 strips / swap
            "pp_slab_square": lambda: ops.wgrad_gemm_pp(dy, x, acc, None, 0, 8),
            "pp_slab_bias_square": lambda: ops.wgrad_gemm_pp(dy, x, acc, bias, 0, 8),
        }
        order = only.replace("+", ",").split(",") if only else list(variants)
        for mode in (0, 8):
            print(json.dumps({"model": model, "M": M, "gemm": name, "plan_mode": mode,
                              **_plan(ops, M, N, K, lda, False, mode)}), flush=True)
        for _ in range(rounds):
            for label in order:
                ms = timeit(variants[label])
                print(json.dumps({"model": model, "M": M, "gemm": name, "variant": label, "ms": round(ms, 4),
                                  "TFLOPs": round(flops / ms / 1e9, 1)}), flush=True)


def _warm(seconds: float = 1.0) -> None:
    """Hold the chip busy before the first timing (the first shape otherwise times at ramping clocks)."""
    import time

    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    t0 = time.time()
    while time.time() - t0 < seconds:
        for _ in range(10):
            a @ a
        torch.cuda.synchronize()


def sweep(model: str, M: int, splits: str, mode: int) -> None:
    """Time each shape at fixed split counts (0 = the planner's choice): where the row-chunk
    quantisation and the slab traffic of the split epilogue cost."""
    ops = _ops()
    _warm()
    first = True
    for name, (N, K) in SHAPES[model].items():
        lda = 50304 if N == 50257 else N
        dy = torch.randn(M, lda, device="cuda", dtype=torch.bfloat16)[:, :N]
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        acc = torch.zeros(N, K, device="cuda")
        flops = 2.0 * M * N * K
        if first:  # the first timing of a process reads high even after _warm (profiles/r5/xl/
            # sweep_split_xl_m32k.jsonl: qkv auto 0.62 ms, the same split later 0.55): time it once, unreported
            timeit(lambda: ops.wgrad_gemm_pp(dy, x, acc, None, 0, mode))
            first = False
        for s in (int(v) for v in splits.replace("+", ",").split(",")):
            ms = timeit(lambda: ops.wgrad_gemm_pp(dy, x, acc, None, s, mode))
            print(json.dumps({"model": model, "M": M, "gemm": name, "split": s, "mode": mode, "ms": round(ms, 4),
                              "TFLOPs": round(flops / ms / 1e9, 1)}), flush=True)


def sweep2(model: str, M: int, splits: str, ssplits: str, gemms: str = "") -> None:
    """Time each shape with tail tiling over (main split, strip split) pairs (0 = planned), the
    256 x 256-only plan first: the data the planner's cost model is checked against."""
    ops = _ops()
    _warm()
    for name, (N, K) in SHAPES[model].items():
        if gemms and name not in gemms.split(","):
            continue
        dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        acc = torch.zeros(N, K, device="cuda")
        flops = 2.0 * M * N * K
        timeit(lambda: ops.wgrad_gemm_pp(dy, x, acc, None, 0, 8))
        ms = timeit(lambda: ops.wgrad_gemm_pp(dy, x, acc, None, 0, 8))
        print(json.dumps({"model": model, "M": M, "gemm": name, "square": True, "ms": round(ms, 4),
                          "TFLOPs": round(flops / ms / 1e9, 1)}), flush=True)
        for sm in (int(v) for v in splits.split(",")):
            for ss in (int(v) for v in ssplits.split(",")):
                sp = sm + 65536 * ss
                plan = ops.wgrad_pp_plan(M, N, K, N, K, False, sp, 0)
                ms = timeit(lambda: ops.wgrad_gemm_pp(dy, x, acc, None, sp, 0))
                print(json.dumps({"model": model, "M": M, "gemm": name, "split": sm, "ssplit": ss, "plan": plan,
                                  "ms": round(ms, 4), "TFLOPs": round(flops / ms / 1e9, 1)}), flush=True)


def one(gemm: str, variant: str, M: int, reps: int) -> None:
    """Run one shape / kernel ``reps`` times (a target for rocprofv3 counter passes)."""
    ops = _ops()
    N, K = {**SHAPES["gpt2-124m"], **SHAPES["head"]}[gemm]
    lda = 50304 if N == 50257 else N
    dy = torch.randn(M, lda, device="cuda", dtype=torch.bfloat16)[:, :N]
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    acc = torch.zeros(N, K, device="cuda")
    fn = {"pp": lambda: ops.wgrad_gemm_pp(dy, x, acc, None, 0, -1)}[variant]
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["check", "time", "one", "sweep", "sweep2"])
    ap.add_argument("--gemm", default="qkv")
    ap.add_argument("--variant", default="pp")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="", help="comma-separated variant labels (time)")
    ap.add_argument("--tokens", type=int, default=131072)
    ap.add_argument("--rounds", type=int, default=1, help="time: repeat the variant sequence")
    ap.add_argument("--model", default="gpt2-124m", choices=sorted(SHAPES))
    ap.add_argument("--splits", default="0,1,2,3,4,5,6,8")
    ap.add_argument("--ssplits", default="0,1,2,4,8,16,32", help="sweep2: strip splits")
    ap.add_argument("--gemms", default="", help="sweep2: comma-separated shape names (default all)")
    ap.add_argument("--mode", type=int, default=0,
                    help="sweep: 0 slabs + finishing launch, 2 atomics, -1 auto")
    args = ap.parse_args()
    if args.what == "check":
        return check()
    if args.what == "sweep2":
        sweep2(args.model, args.tokens, args.splits, args.ssplits, args.gemms)
        return 0
    if args.what == "sweep":
        sweep(args.model, args.tokens, args.splits, args.mode)
        return 0
    if args.what == "one":
        one(args.gemm, args.variant, args.tokens, args.reps)
        return 0
    time_shapes(args.model, args.tokens, args.only, args.rounds)
    return 0


if __name__ == "__main__":
    sys.exit(main())
