#!/bin/bash
# training step kernel profile (current tree) + flash-attention PMC at the bench shape
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3c_prof}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20; tail -1 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o run -- python3 bench.py --no_serve --steps 6 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('bench (traced)', d['ms_per_step'], d['value'])"
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU"
timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/fa_pmc -o run -- python3 lumen/bench/attn_bench.py --B 8 --S 512 --iters 3 > $O/fa_pmc.log 2>&1 || { tail -5 $O/fa_pmc.log; exit 1; }
python3 - $O <<'PY'
import csv, sys, collections, glob
f = glob.glob(sys.argv[1] + "/fa_pmc/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name']
    if 'fa::' not in k: continue
    k = k.split('fa::')[1].split('(')[0]
    agg[k][r['Counter_Name']] += float(r['Counter_Value']); n[(k, r['Counter_Name'])] += 1
for k, d in agg.items():
    c = n[(k, 'SQ_WAVE_CYCLES')]; w = d['SQ_WAVE_CYCLES']
    print(f"{k:42s} active {d['SQ_ACTIVE_INST_ANY']/w:.2f} wait_any {d['SQ_WAIT_ANY']/w:.2f} wait_inst {d['SQ_WAIT_INST_ANY']/w:.2f} (lds {d['SQ_WAIT_INST_LDS']/w:.2f}) mfma_busy/call {d['SQ_VALU_MFMA_BUSY_CYCLES']/c:.3g} bankconf/call {d['SQ_LDS_BANK_CONFLICT']/c:.3g}")
PY
