#!/usr/bin/env python3
"""A/B of the deterministic-mode LM-head logits routing, one process per arm:

    python bench/det_head_ab.py {ours|library} [bench.py args ...]

``ours`` runs ``bench.py`` unchanged (round 6: the logits GEMM on the fixed-order kernel in
deterministic mode); ``library`` first patches :func:`llmtrain.ops.head_logits` back to the
hipBLASLt call of rounds 1-5 (its tuned Stream-K solution).  Pass ``--deterministic`` to bench.py
for the comparison to mean anything; alternate the arms on one box (docs/round6.md §2)."""

from __future__ import annotations

import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    arm = sys.argv[1]
    if arm not in ("ours", "library"):
        raise SystemExit("usage: det_head_ab.py {ours|library} [bench.py args]")
    if arm == "library":
        from llmtrain import ops

        ops.head_logits = lambda h, w: ops._lib_mm(h, w.t(), op="LM-head logits")  # rounds 1-5 routing
    sys.argv = [os.path.join(ROOT, "bench.py"), *sys.argv[2:]]
    runpy.run_path(sys.argv[0], run_name="__main__")


if __name__ == "__main__":
    main()
