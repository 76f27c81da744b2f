#!/usr/bin/env python3
"""GPU busy / idle accounting of the LAST window of a rocprofv3 kernel trace (csv): wall from the
window's first kernel start to its last kernel end, merged kernel-busy time, and the idle time
binned by gap length, with the largest gaps and the kernels around them.

    python scripts/tools/busy_timeline.py gpurun_out/<run>/prof [window_s]"""
import csv
import os
import sys


def main(d, window_s=None):
    f = next(os.path.join(r, n) for r, _, fs in os.walk(d) for n in fs
             if n.endswith("kernel_trace.csv"))
    rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                   for r in csv.DictReader(open(f))))
    if window_s:
        t_end = max(e for _, e, _ in rows)
        rows = [r for r in rows if r[0] >= t_end - window_s * 1e9]
    else:  # after the last idle gap >= 0.3 s
        cut = 0
        end = rows[0][1]
        for i in range(1, len(rows)):
            if rows[i][0] - end >= 300_000_000:
                cut = i
            end = max(end, rows[i][1])
        rows = rows[cut:]
    t0, t1 = rows[0][0], max(e for _, e, _ in rows)
    busy, gaps = 0, []
    cs, ce, prev = rows[0][0], rows[0][1], rows[0][2]
    for s, e, n in rows[1:]:
        if s > ce:
            busy += ce - cs
            gaps.append((s - ce, prev, n))
            cs, ce = s, e
        else:
            ce = max(ce, e)
        prev = n
    busy += ce - cs
    wall = t1 - t0
    print(f"window: {len(rows)} kernels, wall {wall / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms "
          f"({100 * busy / wall:.1f} %), idle {(wall - busy) / 1e6:.2f} ms")
    bins = [(0, 10e3), (10e3, 50e3), (50e3, 200e3), (200e3, 1e6), (1e6, 1e12)]
    for lo, hi in bins:
        g = [x for x, _, _ in gaps if lo <= x < hi]
        print(f"  gaps {lo / 1e3:7.0f}-{hi / 1e3:7.0f} us: {len(g):6d}, {sum(g) / 1e6:8.2f} ms")
    for g, a, b in sorted(gaps, reverse=True)[:12]:
        print(f"  {g / 1e3:9.1f} us  after {a[:50]}  before {b[:50]}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else None)
