#!/bin/bash
# Round 4: kernel stats of the final serving path (prefill_first 4096, engine mode, 256 x 512/128)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_36}; mkdir -p $O
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o serve_pf -- python3 -m lumen.bench.serve_bench \
  --max-model-len 1024 --scheduling-policy prefill_first --max-batched-tokens 4096 > $O/prof_run.json 2> $O/prof_run.err || { tail -20 $O/prof_run.err; exit 1; }
cd $GRAFT_REPO_ROOT
python3 - > $O/kernel_stats.txt <<PY
import csv, glob
f = glob.glob("$O/prof/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"kernel time total {tot/1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} kernels (warm-up round + burst)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    t = float(r["TotalDurationNs"]); n = int(r["Calls"])
    print(f"{t/1e6:9.1f} ms {n:7d} x {t/n/1e3:8.1f} us {100*t/tot:5.1f}%  {r['Name'][:110]}")
PY
head -30 $O/kernel_stats.txt
