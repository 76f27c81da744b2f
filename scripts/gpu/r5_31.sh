#!/bin/bash
# LoRA down3 / dxa3 without serialized guarded loads: numerics, then a traced bench step (per-kernel times)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_31; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "rope or flash or fp32 or qkv" \
  tests/test_production_shapes_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 bench.py --no_serve --partitioned "" --no_comm_probe --steps 20 --warmup 5 > $O/bench_a.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o train -- python3 $GRAFT_REPO_ROOT/bench.py --no_serve --partitioned "" --no_comm_probe --steps 3 --warmup 2 > $O/bench_prof.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cd $GRAFT_REPO_ROOT
python3 - <<PY
import csv, collections, json
d = json.loads(open("$O/bench_a.json").read().strip().splitlines()[-1])
print("bench", d["value"], d["ms_per_step"])
rows = sorted(csv.DictReader(open("$O/prof/train_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "adamw_kernel" in r["Kernel_Name"]]
step = rows[idx[-2] + 1: idx[-1] + 1]
c = collections.defaultdict(list)
for r in step:
    c[r["Kernel_Name"][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(c.items(), key=lambda x: -sum(x[1]))[:24]:
    print(f"{sum(v)/1e3:7.3f} ms {len(v):4d} x {sum(v)/len(v):7.1f} us  {k}")
PY
