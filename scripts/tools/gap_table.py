#!/usr/bin/env python3
"""Kernel table of the work after the LAST idle gap of >= 0.3 s in a rocprofv3 kernel trace (probes
sleep 0.5 s before their timed steps; model loading leaves earlier gaps), grouped by kernel name,
per step.

    python scripts/tools/gap_table.py gpurun_out/<run>/prof STEPS"""
import collections
import csv
import os
import sys


def main(d, steps):
    f = next(os.path.join(r, n) for r, _, fs in os.walk(d) for n in fs
             if n.endswith("kernel_trace.csv"))
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    gaps = [(int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"]), i)
            for i in range(1, len(rows))]
    first = max(i for g, i in gaps if g >= 300_000_000) if any(g >= 300_000_000 for g, _ in gaps) \
        else max(gaps)[1]
    seg = rows[first:]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    c = collections.defaultdict(lambda: [0, 0])
    for r in seg:
        k = r["Kernel_Name"][:100]
        c[k][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        c[k][1] += 1
    tot = sum(v[0] for v in c.values())
    print(f"steps: {steps}, wall {(t1 - t0) / 1e6 / steps:.3f} ms/step, kernel sum "
          f"{tot / 1e6 / steps:.3f} ms/step, {len(seg) / steps:.0f} launches/step")
    for k, v in sorted(c.items(), key=lambda x: -x[1][0]):
        print(f"{v[0] / 1e6 / steps:8.3f} ms/step {v[1] / steps:6.1f} x {v[0] / v[1] / 1e3:8.1f} us  {k}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
