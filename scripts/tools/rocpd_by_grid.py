"""Per-(kernel, grid) call count and mean us from a rocpd database (kernels with the same name
but different grids, e.g. the q|k|v and o launches of one LoRA kernel, apart).

    python3 scripts/tools/rocpd_by_grid.py <dir or .db> <name filter>"""
import collections
import glob
import os
import sqlite3
import sys

path, filt = sys.argv[1], sys.argv[2]
dbs = [path] if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
for f in dbs:
    c = sqlite3.connect(f)
    t = collections.defaultdict(list)
    for n, gx, gy, gz, d in c.execute("select name, grid_x, grid_y, grid_z, end - start from kernels"):
        if filt in n:
            t[(n[:70], gx, gy, gz)].append(d)
    for (n, gx, gy, gz), v in sorted(t.items()):
        print(f"{len(v):5d} x {sum(v) / len(v) / 1e3:8.2f} us  grid {gx}x{gy}x{gz}  {n}")
