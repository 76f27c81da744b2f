#!/bin/bash
# FA iteration: numerics tests, attn_bench at the training shape, one PMC pass (conflicts / waits)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r2_fa}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "flash or llama_layer" --timeout 120 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 120 python lumen/bench/attn_bench.py --B 8 --S 512 --iters 50 > $O/attn_$i.json 2>&1 || exit 1
tail -1 $O/attn_$i.json
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 lumen/bench/attn_bench.py --only ${FA_ONLY:-all} --B 8 --S 512 --iters 20 > $O/kt.log 2>&1 || exit 1
python3 - $(find $O/kt -name "*kernel_stats.csv" | head -1) <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "lumen" in r["Name"]:
        print(f'{float(r["AverageNs"])/1e3:8.1f} us  x{r["Calls"]:>4}  {r["Name"][:80]}')
PY
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $C1 --output-format csv -d $O/pmc_1 -o run -- python3 lumen/bench/attn_bench.py --only bwd --B 8 --S 512 --iters 3 > $O/pmc_1.log 2>&1 || exit 1
python3 - $O/pmc_1/run_counter_collection.csv <<'PY'
import csv, collections, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "lumen::fa" not in n: continue
    agg[n.split("(")[0].replace("void lumen::fa::", "")][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    wc = d["SQ_WAVE_CYCLES"]
    print(k, " ".join(f"{c[3:]}={d[c]/wc:.3f}" for c in sorted(d) if c.startswith("SQ_WAIT") or c.startswith("SQ_ACTIVE")),
          f"conflict/lds={d['SQ_LDS_BANK_CONFLICT']/max(d['SQ_LDS_IDX_ACTIVE'],1):.3f}")
PY
