#!/usr/bin/env python3
"""A/B of the weight-gradient tail tiling (csrc/gemm_wgrad_pp.hip), one process per arm:

    python bench/wgrad_tail_ab.py {tails|square} [bench.py args ...]

``tails`` runs ``bench.py`` unchanged (round 6: 512 x 64 strip tiles for a K tail, swapped operands
for an N tail); ``square`` first patches :func:`llmtrain.ops.wgrad_accum` to the 256 x 256-only
plan of rounds 1-5 (the op's mode + 8).  Only shapes whose N or K is not a multiple of 256 differ
(GPT-2 XL's d = 1600); alternate the arms on one box (docs/round6.md §10)."""

from __future__ import annotations

import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    arm = sys.argv[1]
    if arm not in ("tails", "square"):
        raise SystemExit("usage: wgrad_tail_ab.py {tails|square} [bench.py args]")
    if arm == "square":
        from llmtrain import ops

        tails = ops.wgrad_accum

        def square(dst, dy, x, *, bias=None):
            if not ops._on_gpu(dst):
                return tails(dst, dy, x, bias=bias)
            ops.hip_ops().wgrad_gemm_pp(dy, x, dst, bias, 0, 7)  # mode -1 + 8: auto, square tiles only

        ops.wgrad_accum = square
    sys.argv = [os.path.join(ROOT, "bench.py"), *sys.argv[2:]]
    runpy.run_path(sys.argv[0], run_name="__main__")


if __name__ == "__main__":
    main()
