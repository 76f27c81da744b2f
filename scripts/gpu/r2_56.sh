#!/bin/bash
# ZeRO-3 schedules with forced partitioning at world 1 (the N>1 code path) on the current kernels,
# plus a torch profiler op table of the release schedule
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r2_56; mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/id.json 2> $O/id.err || exit $?
python -c "import json;d=json.load(open('$O/id.json'));print('identity', d['ms_per_step'], d['extra']['peak_hbm_gb_max_rank'])"
for sch in pipelined keep; do
  LUMEN_ZERO3_SINGLE=1 LUMEN_ZERO3_SCHEDULE=$sch timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/$sch.json 2> $O/$sch.err || exit $?
  python -c "import json;d=json.load(open('$O/$sch.json'));print('$sch', d['ms_per_step'], d['extra']['peak_hbm_gb_max_rank'], d['extra']['zero3_exposed_wait_ms_per_step_max_rank'])"
done
LUMEN_ZERO3_SINGLE=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config configs/ds_config_zero3_release.json > $O/release.json 2> $O/release.err || exit $?
python -c "import json;d=json.load(open('$O/release.json'));print('release', d['ms_per_step'], d['extra']['peak_hbm_gb_max_rank'], d['extra']['zero3_exposed_wait_ms_per_step_max_rank'], d['extra']['zero3'])"
LUMEN_ZERO3_SINGLE=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o rel --output-format csv -- python3 bench.py --steps 4 --warmup 2 --config configs/ds_config_zero3_release.json > $O/prof_rel.json 2> $O/prof_rel.log || exit $?
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{float(r["TotalDurationNs"]) / 6e6:8.3f} ms/step {r["Calls"]:>5}  {r["Name"][:90]}')
PY
