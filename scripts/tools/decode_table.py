#!/usr/bin/env python3
"""Kernel table of the decode steps of scripts/probes/decode_step_probe.py from a rocprofv3
kernel trace: the kernels after the largest idle gap (the probe sleeps 0.5 s before its timed
decode steps), grouped by name, per step (n_steps = pa_decode launches / layers).

    python scripts/tools/decode_table.py gpurun_out/<run>/prof [layers=32]"""
import collections
import csv
import os
import sys


def main(d, layers=32):
    f = next(os.path.join(r, n) for r, _, fs in os.walk(d) for n in fs
             if n.endswith("kernel_trace.csv"))
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    # decode steps = everything after the last prefill kernel (flash-attention prefill or a
    # 256 x 256 macro-tile prefill GEMM), from the first paged-decode launch on
    last_pf = max((i for i, r in enumerate(rows)
                   if "fwd32_kernel" in r["Kernel_Name"] or "MT256x256" in r["Kernel_Name"]),
                  default=-1)
    first = next(i for i in range(last_pf + 1, len(rows)) if "pa_decode" in rows[i]["Kernel_Name"])
    # start at the first kernel of that step: back up to the step's first RMSNorm / embedding
    while first > last_pf + 1 and "embedding" not in rows[first - 1]["Kernel_Name"]:
        first -= 1
    seg = rows[first:]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    c = collections.defaultdict(lambda: [0, 0])
    for r in seg:
        k = r["Kernel_Name"][:90]
        c[k][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        c[k][1] += 1
    npa = sum(v[1] for k, v in c.items() if "pa_decode" in k)
    steps = max(1, npa // layers)
    tot = sum(v[0] for v in c.values())
    print(f"decode steps: {steps}, wall {(t1 - t0) / 1e6 / steps:.3f} ms/step, kernel sum "
          f"{tot / 1e6 / steps:.3f} ms/step, {len(seg) / steps:.0f} launches/step")
    for k, v in sorted(c.items(), key=lambda x: -x[1][0]):
        print(f"{v[0] / 1e6 / steps:8.3f} ms/step {v[1] / steps:5.1f} x {v[0] / v[1] / 1e3:7.1f} us  {k}")


if __name__ == "__main__":
    main(sys.argv[1], *(int(x) for x in sys.argv[2:]))
