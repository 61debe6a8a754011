"""Can a bandwidth-bound kernel hide under a GEMM on another stream?  Times a hipBLASLt GEMM and
a group of memory-bound kernels (add+LayerNorm forward, GELU forward, cross-entropy) alone and
issued concurrently on two HIP streams, at half-micro-batch shapes (M = 65536 tokens).

    python bench/overlap.py
"""

from __future__ import annotations

import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def timed(fn, reps: int = 10) -> float:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main() -> None:
    from llmtrain.ops import _ext

    _ext.require()
    ops = torch.ops.llmtrain_hip
    dev = torch.device("cuda")
    M, d = 65536, 768
    bf = torch.bfloat16
    h = torch.randn(M, d, device=dev, dtype=bf)
    w_fc = torch.randn(4 * d, d, device=dev, dtype=bf) * 0.02
    b_fc = torch.zeros(4 * d, device=dev, dtype=bf)
    w_qkv = torch.randn(3 * d, d, device=dev, dtype=bf) * 0.02
    x = torch.randn(M, d, device=dev)
    delta = torch.randn(M, d, device=dev, dtype=bf)
    lw, lb = torch.ones(d, device=dev), torch.zeros(d, device=dev)
    u = torch.randn(M, 4 * d, device=dev, dtype=bf)
    logits = torch.randn(M // 4, 50304, device=dev, dtype=bf)
    labels = torch.randint(0, 50257, (M // 4,), device=dev)
    roww = torch.full((M // 4,), 1.0 / M, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def gemm():
        torch.addmm(b_fc, h, w_fc.t())
        torch.mm(h, w_qkv.t())

    def mem():
        ops.add_layernorm_fwd(x, delta, lw, lb, 1e-5, bf)
        ops.gelu_fwd(u)
        ops.cross_entropy_fwd_bwd(logits, labels, 50257, roww)

    def both():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            gemm()
        with torch.cuda.stream(s2):
            mem()
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    tg, tm, tb = timed(gemm), timed(mem), timed(both)
    print(json.dumps({"gemm_ms": round(tg, 3), "mem_ms": round(tm, 3), "sum_ms": round(tg + tm, 3),
                      "concurrent_ms": round(tb, 3), "hidden_fraction_of_mem": round((tg + tm - tb) / tm, 3)}))


if __name__ == "__main__":
    main()
