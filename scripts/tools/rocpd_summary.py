"""Summarise a rocprofv3 rocpd database (the default output format of this ROCm): per-kernel
call count / mean / min us from ``kernels``, and per-kernel mean counter values from
``counters_collection``.

    python3 scripts/tools/rocpd_summary.py <dir or .db> [name filter]
"""
import collections
import glob
import os
import sqlite3
import sys


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    dbs = [path] if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"),
                                                            recursive=True)
    for f in dbs:
        c = sqlite3.connect(f)
        t = collections.defaultdict(list)
        for n, d in c.execute("select name, end - start from kernels"):
            if filt in n:
                t[n].append(d)
        for n, v in sorted(t.items(), key=lambda kv: -sum(kv[1])):
            print(f"{len(v):5d} x {sum(v) / len(v) / 1e3:9.2f} us (min {min(v) / 1e3:8.2f})  {n[:90]}")
        cnt = collections.defaultdict(list)
        try:
            for n, cn, v in c.execute("select kernel_name, counter_name, value from counters_collection"):
                if filt in n:
                    cnt[(n, cn)].append(v)
        except sqlite3.OperationalError:
            pass
        for (n, cn), v in sorted(cnt.items()):
            print(f"  {cn:28s} {sum(v) / len(v):16.1f}  ({len(v)} dispatches)  {n[:60]}")


if __name__ == "__main__":
    main()
