#!/usr/bin/env python3
"""Summarise a rocprofv3 *_kernel_stats.csv as per-step times: kstats.py CSV STEPS [TOP]."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:top]:
    ms = float(r["TotalDurationNs"]) / 1e6 / steps
    print(f"{ms:7.2f} ms/step {int(r['Calls']) / steps:6.1f}/step {float(r['AverageNs']) / 1e3:8.1f} us  {r['Name'][:90]}")
print(f"total {tot / 1e6 / steps:.2f} ms/step")
