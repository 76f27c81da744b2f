#!/bin/bash
# batch-1 GEMV forms + SwiGLU fusion microbench, then the decode A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-s3_gemv}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "skinny or swiglu or paged" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u lumen/bench/skinny_bench.py --m1-forms > $O/m1_forms.jsonl 2>&1 || exit 1
cat $O/m1_forms.jsonl
bash scripts/gpu/s3_pa_ab.sh ${1:-s3_gemv}
