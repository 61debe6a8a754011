#!/usr/bin/env python3
"""Per-step kernel summary from a rocprofv3 SQLite trace (``run_results.db``).

    python scripts/rocpd_stats.py gpurun_out/prof/run_results.db [SKIP_STEPS] [TOP]

Step boundaries are the AdamW kernel (one per optimizer step); the first SKIP_STEPS steps
(warm-up, default 3) are dropped.  Prints ms/step per kernel, per-stream busy time and the
wall time per step (AdamW end to AdamW end).
"""

from __future__ import annotations

import sqlite3
import sys
from collections import defaultdict


def main() -> None:
    db = sys.argv[1]
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    con = sqlite3.connect(db)
    rows = con.execute("select name, stream_id, start, end from kernels order by start").fetchall()
    marks = [r[3] for r in rows if "adamw_kernel" in r[0] or "adamw_tiled_kernel" in r[0]]
    if len(marks) <= skip + 1:
        raise SystemExit(f"only {len(marks)} optimizer steps in the trace")
    t0, t1 = marks[skip], marks[-1]
    steps = len(marks) - 1 - skip
    per = defaultdict(lambda: [0, 0])
    busy = defaultdict(int)
    for name, stream, s, e in rows:
        if s < t0 or e > t1:
            continue
        per[name][0] += e - s
        per[name][1] += 1
        busy[stream] += e - s
    total = sum(v[0] for v in per.values())
    for name, (ns, n) in sorted(per.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"{ns / 1e6 / steps:7.2f} ms/step {n / steps:6.1f}/step {ns / n / 1e3:8.1f} us  {name[:96]}")
    print(f"kernel time {total / 1e6 / steps:.2f} ms/step over {steps} steps; wall {(t1 - t0) / 1e6 / steps:.2f} ms/step")
    for stream, ns in sorted(busy.items(), key=lambda kv: -kv[1]):
        print(f"  stream {stream}: busy {ns / 1e6 / steps:.2f} ms/step")


if __name__ == "__main__":
    main()
