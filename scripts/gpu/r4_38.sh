#!/bin/bash
# Round 4: decode RMSNorm A/B -- workgroup-per-row kernel (default below 1024 rows) vs the
# multi-row kernel at the 256-row decode step (LUMEN_RMS_ROW_MAX=128)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_38}; mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k rmsnorm > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -n 1 $O/tests.txt
B="python -m lumen.bench.serve_bench --max-model-len 1024 --scheduling-policy prefill_first --max-batched-tokens 4096 --trace-steps"
for v in 1024 128 1024; do
  LUMEN_RMS_ROW_MAX=$v timeout -k 10 300 $B > $O/rm$v.json 2> $O/rm$v.err || { tail -5 $O/rm$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/rm$v.json').read().strip().splitlines()[-1]); st=d['step_trace']
print('row_max $v', d['output_tok_s'], st['decode']['ms_mean'], st['prefill']['ms_mean'])"
done
