#!/bin/bash
# flash-attention diagnosis: per-shape forward/backward timing and PMC of the forward kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_fa_diag}; mkdir -p $O
timeout -k 10 180 python3 scripts/probes/fa_fwd_probe.py --bwd > $O/shapes.jsonl 2> $O/shapes.err || { tail -5 $O/shapes.err; exit 1; }
cat $O/shapes.jsonl
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
  --output-format csv -d $O/pmc1 -o run -- python3 scripts/probes/fa_fwd_probe.py --shapes 8x512c,2x2048n --iters 3 > $O/pmc1.log 2>&1 || { tail -5 $O/pmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU \
  --output-format csv -d $O/pmc2 -o run -- python3 scripts/probes/fa_fwd_probe.py --shapes 8x512c,2x2048n --iters 3 > $O/pmc2.log 2>&1 || { tail -5 $O/pmc2.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys, collections
for p in ("pmc1", "pmc2"):
    fs = glob.glob(f"{sys.argv[1]}/{p}/**/*counter_collection.csv", recursive=True)
    if not fs:
        print("no csv for", p); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(fs[0])):
        n = r["Kernel_Name"]
        if "lumen::fa" not in n:
            continue
        key = (n[:60], r.get("Grid_Size", ""))
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        print(p, k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
