#!/bin/bash
# library GEMMs of the training step: clock and MFMA busy from a counter pass (+ plain timing)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_44; mkdir -p $O
timeout -k 10 120 python3 scripts/probes/gemm_pmc.py > $O/timing.txt 2>&1 || { tail -5 $O/timing.txt; exit 1; }
cat $O/timing.txt
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -d $O/pmc -o pmc -- python3 scripts/probes/gemm_pmc.py > $O/pmc_run.txt 2>&1 || { tail -5 $O/pmc_run.txt; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/kt -o kt -- python3 scripts/probes/gemm_pmc.py > $O/kt_run.txt 2>&1 || { tail -5 $O/kt_run.txt; exit 1; }
python3 - <<PY
import sqlite3, glob, collections
c = sqlite3.connect(glob.glob("$O/pmc/*.db")[0])
rows = c.execute("select dispatch_id, kernel_name, counter_name, value, grid_size from counters_collection").fetchall()
d = collections.defaultdict(dict)
for did, n, cn, v, g in rows:
    d[did][cn] = v; d[did]["name"] = n; d[did]["grid"] = g
k = sqlite3.connect(glob.glob("$O/kt/*.db")[0])
kt = [(n, (e - s)) for n, s, e in k.execute("select name, start, end from kernels order by start")]
pm = [d[i] for i in sorted(d)]
print("dispatches", len(pm), len(kt))
for (n, dur), p in zip(kt, pm):
    if "Cijk" not in n and "gemm" not in n.lower():
        continue
    ga = p.get("GRBM_GUI_ACTIVE", 0)
    print(f"{dur/1e3:8.1f} us  clk~{ga / dur:5.2f} GHz  mfma_busy {p.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (1024 * max(ga, 1)):5.2f}  {n[:70]}")
PY
# serving burst (in-process engine, prefill-first 4096, the bench's settings): GPU busy / idle
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/serve -o serve -- python3 -m lumen.bench.serve_bench --mode engine --scheduling-policy prefill_first --max-batched-tokens 4096 --max-model-len 1024 > $O/serve.json 2> $O/serve.err || { tail -20 $O/serve.err; exit 1; }
tail -2 $O/serve.json
python3 scripts/tools/busy_timeline.py $O/serve 3.9
