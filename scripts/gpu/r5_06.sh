#!/bin/bash
# paged decode v1 vs v2 kernel traces, fp8 KV A/B, then the full bench record on this tree
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5_06
LUMEN_PA_1PASS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_06/prof_v1 -o dec --output-format csv -- python3 scripts/probes/decode_step_probe.py > gpurun_out/r5_06/prof_v1.log 2>&1 || exit 1
python3 scripts/tools/decode_table.py gpurun_out/r5_06/prof_v1 > gpurun_out/r5_06/decode_table_v1.txt
for v in 2 1; do
  LUMEN_PA_1PASS=$v timeout -k 10 300 python -u scripts/probes/decode_step_probe.py --kv fp8 >> gpurun_out/r5_06/fp8_v$v.txt 2>&1 || exit 1
done
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/r5_06/bench.json 2> gpurun_out/r5_06/bench.err || { tail -20 gpurun_out/r5_06/bench.err; exit 1; }
head -8 gpurun_out/r5_06/decode_table_v1.txt; grep -h ms_per gpurun_out/r5_06/fp8_v*.txt
python3 -c "
import json; j=json.load(open('gpurun_out/r5_06/bench.json')); x=j['extra']
print('train', j['value'], j['ms_per_step'])
for k in ('serve','serve_engine','serve_chunked'):
    s=x.get(k) or {}; print(k, s.get('output_tok_s'), s.get('ttft_p50_ms'), s.get('itl_p50_ms'), s.get('itl_p99_ms'))
"
