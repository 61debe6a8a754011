"""Run-to-run bitwise check of the library's Stream-K GEMM solutions (the `..._SK3_...` kernels).

    python bench/sk_repeat.py [reps]

The LM-head logits GEMM (M x 768 @ 768 x 50304) and the forward projections, issued exactly as the
trainer issues them (shipped TunableOp table), ``reps`` times on identical inputs — alone, and with
a second stream running an unrelated GEMM so the workgroups finish in a different order.  Every
output is compared bitwise with the first.  One JSON line per case.
"""

from __future__ import annotations

import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main() -> int:
    from llmtrain.runtime.tuning import enable_tuned_gemms

    enable_tuned_gemms(torch.device("cuda"))
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    g = torch.Generator(device="cuda").manual_seed(0)
    bf = dict(device="cuda", dtype=torch.bfloat16)

    def rnd(*shape, scale=1.0):
        return (torch.randn(*shape, device="cuda", generator=g) * scale).to(torch.bfloat16)

    cases = {}
    for m in (8192, 32768):
        h, w = rnd(m, 768), rnd(50304, 768, scale=0.02)
        cases[f"LM-head logits M={m}"] = (lambda h=h, w=w: torch.mm(h, w.t()))
    x = rnd(131072, 768)
    wq, bq = rnd(2304, 768, scale=0.02), torch.randn(2304, **bf)
    cases["qkv forward M=131072 (addmm)"] = lambda: torch.addmm(bq, x, wq.t())
    xp = rnd(16384, 6400)
    wp, bp = rnd(1600, 6400, scale=0.02), torch.randn(1600, **bf)
    cases["XL proj forward M=16384 (addmm)"] = lambda: torch.addmm(bp, xp, wp.t())

    side = torch.cuda.Stream()
    a = rnd(4096, 4096)
    bad = 0
    for name, fn in cases.items():
        for loaded in (False, True):
            ref = fn().clone()
            diff = 0
            for _ in range(reps):
                if loaded:
                    with torch.cuda.stream(side):
                        for _ in range(2):
                            a @ a
                y = fn()
                diff += int(not torch.equal(y, ref))
            torch.cuda.synchronize()
            bad += diff
            print(json.dumps({"case": name, "concurrent_load": loaded, "reps": reps, "differing": diff}), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
