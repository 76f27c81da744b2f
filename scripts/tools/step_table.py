#!/usr/bin/env python3
"""Per-step kernel table from a rocprofv3 kernel trace: the last complete optimizer step (between
the last two fused-AdamW launches), grouped by kernel name, plus wall vs busy time.

    python scripts/tools/step_table.py gpurun_out/<run>/prof > table.txt"""
import collections
import csv
import os
import sys


def main(d):
    f = next(os.path.join(r, n) for r, _, fs in os.walk(d) for n in fs
             if n.endswith("kernel_trace.csv"))
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    ad = [i for i, r in enumerate(rows) if "adamw_kernel" in r["Kernel_Name"]]
    seg = rows[ad[-2] + 1:ad[-1] + 1]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    c = collections.defaultdict(lambda: [0, 0])
    for r in seg:
        k = r["Kernel_Name"][:80]
        c[k][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        c[k][1] += 1
    tot = sum(v[0] for v in c.values())
    print(f"one steady-state step: wall {(t1 - t0) / 1e6:.2f} ms, kernel sum {tot / 1e6:.2f} ms, "
          f"{len(seg)} launches")
    for k, v in sorted(c.items(), key=lambda x: -x[1][0]):
        print(f"{v[0] / 1e6:8.3f} ms {v[1]:4d} x {v[0] / v[1] / 1e3:7.1f} us  {k}")


if __name__ == "__main__":
    main(sys.argv[1])
