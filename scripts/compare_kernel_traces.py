import csv, sys, collections
def load(path, warm_steps=2, layers=32):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # find start of timed region: the (warm_steps*layers+1)-th fa fwd kernel
    fa = [i for i, r in enumerate(rows) if "fa::fwd" in r["Kernel_Name"]]
    start = fa[warm_steps * layers]
    # back up to the embedding gather before it? approximate: from start
    tl = rows[start:]
    t0 = int(tl[0]["Start_Timestamp"]); t1 = max(int(r["End_Timestamp"]) for r in tl)
    agg = collections.defaultdict(lambda: [0, 0])
    streams = collections.defaultdict(int)
    for r in tl:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        n = r["Kernel_Name"]
        key = ("GEMM " + n[:40]) if ("Cijk" in n) else n[:90]
        agg[key][0] += d; agg[key][1] += 1
        streams[r["Queue_Id"]] += d
    return agg, (t1 - t0), streams
a, wa, sa = load(sys.argv[1]); b, wb, sb = load(sys.argv[2])
steps = 5
print(f"wall {wa/1e6/steps:.2f} vs {wb/1e6/steps:.2f} ms/step; queues {dict(sa)} | {dict(sb)}")
keys = sorted(set(a) | set(b), key=lambda k: -(b.get(k, [0])[0] + a.get(k, [0])[0]))
tot_a = tot_b = 0
for k in keys[:40]:
    x = a.get(k, [0, 0]); y = b.get(k, [0, 0])
    tot_a += x[0]; tot_b += y[0]
    print(f"{x[0]/1e6/steps:8.2f} {y[0]/1e6/steps:8.2f} ms  {x[1]//steps:5d} {y[1]//steps:5d}  {k}")
print("sum", sum(v[0] for v in a.values())/1e6/steps, sum(v[0] for v in b.values())/1e6/steps)
