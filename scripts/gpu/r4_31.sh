#!/bin/bash
# Round 4: weight-streaming decode GEMM -- numerics first (fp32 reference), then the probe
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4_31}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wsgemm_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -n 2 $O/tests.txt
timeout -k 10 400 python scripts/probes/wsg_probe.py > $O/probe.jsonl 2> $O/probe.err || { tail -10 $O/probe.err; exit 1; }
python3 -c "
import json
for l in open('$O/probe.jsonl'):
    d = json.loads(l); d.pop('sweep', None); print(d)"
