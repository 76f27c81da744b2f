#!/bin/bash
# FA forward cost split at B=8 S=512 causal (LUMEN_FA_PROBE 0 / 1 = no tile math / 2 = no K/V
# loads) + one counter pass (HBM fetch bytes, MFMA busy) on the production kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_38; mkdir -p $O
for p in 0 1 2; do
  LUMEN_FA_PROBE=$p timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p$p -o p$p -- \
    python3 lumen/bench/attn_bench.py --only fwd --iters 30 > $O/p$p.json 2> $O/p$p.err || exit 1
done
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d $O/pmc -o pmc -- \
  python3 lumen/bench/attn_bench.py --only fwd --iters 10 > $O/pmc.json 2> $O/pmc.err || exit 1
python3 - <<PY
import csv, glob, collections
for p in (0, 1, 2):
    f = glob.glob("$O/p%d/**/*kernel_stats.csv" % p, recursive=True)
    for r in csv.DictReader(open(f[0])):
        if "fwd32" in r["Name"]:
            print("probe", p, r["Calls"], "avg us", round(float(r["AverageNs"]) / 1e3, 2), r["Name"][:70])
f = glob.glob("$O/pmc/**/*counter_collection.csv", recursive=True)
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f[0])):
    if "fwd32" in r["Kernel_Name"]:
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(k, len(v), sum(v) / len(v))
PY
