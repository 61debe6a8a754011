#!/usr/bin/env python3
"""One optimizer step's kernel timeline from a rocprofv3 SQLite trace, plus a phase summary.

    python scripts/rocpd_timeline.py run_results.db [STEP_INDEX]

Prints every kernel of the chosen step (AdamW end to AdamW end) in start order with its stream,
start offset and duration, then per-stream busy time split into forward (before the
cross-entropy kernel ends) and backward, so each GEMM can be attributed to its op.
"""

from __future__ import annotations

import sqlite3
import sys
from collections import defaultdict


def main() -> None:
    db = sys.argv[1]
    idx = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    con = sqlite3.connect(db)
    rows = con.execute("select name, stream_id, start, end from kernels order by start").fetchall()
    marks = [r[3] for r in rows if "adamw_kernel" in r[0] or "adamw_tiled_kernel" in r[0]]
    t0, t1 = marks[idx], marks[idx + 1]
    step = [r for r in rows if r[2] >= t0 and r[3] <= t1]
    ce_end = next((e for n, _, _, e in step if "ce_fwd_bwd" in n), t0)
    phase = defaultdict(float)
    for name, stream, s, e in step:
        ph = "fwd" if e <= ce_end else "bwd"
        phase[(stream, ph)] += (e - s) / 1e6
        print(f"{(s - t0) / 1e3:10.1f} us  {(e - s) / 1e3:8.1f} us  s{stream}  {ph}  {name[:110]}")
    print(f"step wall {(t1 - t0) / 1e6:.2f} ms; forward ends at {(ce_end - t0) / 1e6:.2f} ms")
    for (stream, ph), ms in sorted(phase.items()):
        print(f"  stream {stream} {ph}: busy {ms:.2f} ms")


if __name__ == "__main__":
    main()
