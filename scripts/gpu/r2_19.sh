#!/bin/bash
# FA at the training shape (B=8, S=512, 32 heads): per-kernel times + PMC (MFMA busy, waits)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2_19}; mkdir -p $O
timeout -k 10 120 python lumen/bench/attn_bench.py --B 8 --S 512 > $O/attn.json 2> $O/attn.err || exit $?
cat $O/attn.json
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/pmc -o run -- python3 lumen/bench/attn_bench.py --B 8 --S 512 --iters 3 > $O/pmc.log 2>&1 || exit $?
f=$(find $O/pmc -name "*counter_collection.csv" | head -1)
python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    if "fa::" not in k:
        continue
    wc = d["SQ_WAVE_CYCLES"] or 1
    n = cnt[(k, "SQ_WAVE_CYCLES")]
    print(k, "dispatches", n)
    print("   wait_any %.2f wait_inst %.2f active %.2f | mfma_busy/busy %.3f | valu/wave %.0f | gui_active/disp %.0f" % (
        d["SQ_WAIT_ANY"] / wc, d["SQ_WAIT_INST_ANY"] / wc, d["SQ_ACTIVE_INST_ANY"] / wc,
        d["SQ_VALU_MFMA_BUSY_CYCLES"] / max(d["SQ_BUSY_CYCLES"], 1) / 4,
        d["SQ_INSTS_VALU"] / max(d["SQ_WAVES"], 1), d["GRBM_GUI_ACTIVE"] / max(n, 1)))
PY
