#!/usr/bin/env python3
"""Memory traffic per kernel from rocprofv3 counter passes: FETCH_SIZE (L2 reads from the memory
fabric, KiB) and WRITE_SIZE (KiB) per dispatch, joined with the kernel trace of the same run for
durations; grouped by kernel name over the last complete optimizer step (between the last two
fused-AdamW launches).  Prints time, MB moved and the achieved GB/s per kernel.

    python scripts/tools/pmc_bw.py gpurun_out/<run>/fetch gpurun_out/<run>/write > table.txt"""
import collections
import csv
import os
import sys


def _find(d, suffix):
    return next(os.path.join(r, n) for r, _, fs in os.walk(d) for n in fs if n.endswith(suffix))


def _pass(d, counter):
    """{dispatch id: (kernel name, ns, value KiB)} of the last step of one counter pass."""
    trace = sorted(csv.DictReader(open(_find(d, "kernel_trace.csv"))),
                   key=lambda r: int(r["Start_Timestamp"]))
    ad = [i for i, r in enumerate(trace) if "adamw_kernel" in r["Kernel_Name"]]
    seg = trace[ad[-2] + 1:ad[-1] + 1]
    dur = {r["Dispatch_Id"]: (r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
           for r in seg}
    val = collections.defaultdict(float)
    for r in csv.DictReader(open(_find(d, "counter_collection.csv"))):
        if r["Counter_Name"] == counter and r["Dispatch_Id"] in dur:
            val[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: (n, t, val.get(k, 0.0)) for k, (n, t) in dur.items()}


def main(fetch_dir, write_dir):
    f = _pass(fetch_dir, "FETCH_SIZE")
    w = _pass(write_dir, "WRITE_SIZE")
    agg = collections.defaultdict(lambda: [0, 0, 0.0, 0, 0.0])  # n, ns(fetch run), KiB r, ns(w), KiB w
    for _, (n, t, v) in f.items():
        a = agg[n[:70]]
        a[0] += 1
        a[1] += t
        a[2] += v
    for _, (n, t, v) in w.items():
        a = agg[n[:70]]
        a[3] += t
        a[4] += v
    tot = sum(a[1] for a in agg.values())
    print(f"last step of the FETCH_SIZE pass: kernel sum {tot / 1e6:.2f} ms (counter passes "
          f"serialise dispatches: times are per kernel, not the step's wall)")
    print(f"{'ms':>8} {'calls':>5} {'us/call':>8} {'read MB':>8} {'write MB':>8} {'GB/s':>7}  kernel")
    for k, a in sorted(agg.items(), key=lambda x: -x[1][1]):
        if not a[0]:
            continue
        us = a[1] / a[0] / 1e3
        rmb = a[2] / a[0] * 1024 / 1e6
        wmb = a[4] / max(1, a[0]) * 1024 / 1e6
        gbs = (rmb + wmb) / us * 1e3 if us else 0.0
        print(f"{a[1] / 1e6:8.3f} {a[0]:5d} {us:8.1f} {rmb:8.1f} {wmb:8.1f} {gbs:7.0f}  {k}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
