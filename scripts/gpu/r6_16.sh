#!/bin/bash
# sampler kernel durations (rocprofv3 kernel trace) per configuration of the probe
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6_16; mkdir -p $O
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o kt -- python3 scripts/probes/sampler_probe.py > $O/sampler.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
python3 - <<PY
import csv
rows=[r for r in csv.DictReader(open("$O/prof/kt_kernel_trace.csv")) if "sample_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r:int(r["Start_Timestamp"]))
names=[f"s{s}_{n}" for s in (1,3,8) for n in ("greedy","topk50","topp0.95","both")]
for i,n in enumerate(names):
    ch=rows[i*53:(i+1)*53][3:]
    d=sorted((int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1000 for r in ch)
    print(n, "kernel us med", round(d[len(d)//2],1))
PY
