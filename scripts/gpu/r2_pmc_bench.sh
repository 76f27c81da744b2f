#!/bin/bash
# PMC pass over the 1-GPU training step: LDS bank conflicts and wave wait ratios per lumen kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r2_pmc}; mkdir -p $O
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE"
timeout -s KILL 300 rocprofv3 --pmc $C1 --output-format csv -d $O/pmc -o run -- python3 bench.py --steps 1 --warmup 1 > $O/pmc.log 2>&1 || exit 1
python3 - $O/pmc/run_counter_collection.csv > $O/summary.txt <<'PY'
import csv, collections, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "lumen" not in n: continue
    agg[n.split("(")[0].replace("void lumen::", "")[:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in sorted(agg.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"]):
    wc = d["SQ_WAVE_CYCLES"]
    print(f"{k:60s} wc={wc:.3g} " + " ".join(f"{c[3:]}={d[c]/wc:.3f}" for c in sorted(d) if c.startswith("SQ_WAIT") or c.startswith("SQ_ACTIVE")),
          f"conflict/lds={d['SQ_LDS_BANK_CONFLICT']/max(d['SQ_LDS_IDX_ACTIVE'],1):.3f}")
PY
cat $O/summary.txt
