#!/bin/bash
# round-3 re-entry closing measurements: driver-command bench (train + extra.serve), a traced
# steady-state step table, OpenAI HTTP serving
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3d_final}; mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
timeout -k 10 300 python bench.py --no_serve --steps 20 --warmup 5 > $O/bf16.json 2> $O/bf16.err || { tail -5 $O/bf16.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bf16.json'));print('bf16 20 steps', d['ms_per_step'], d['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o run -- python3 bench.py --no_serve --steps 4 --warmup 3 > $O/traced.json 2> $O/traced.err || { tail -5 $O/traced.err; exit 1; }
python3 scripts/tools/step_table.py $O/step > $O/step_table.txt && head -40 $O/step_table.txt
timeout -k 10 400 python -m lumen.bench.serve_bench --mode http > $O/http.json 2> $O/http.err || { tail -5 $O/http.err; exit 1; }
tail -1 $O/http.json
