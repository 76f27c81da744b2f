#!/bin/bash
# decode-batch MFMA GEMM: numerics, per-shape sweep vs hipBLASLt, serving A/B (engine)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3c_bg}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -k "batch_gemm or skinny" --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; grep -E "FAILED|^E " $O/tests.txt | head -20; tail -1 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m lumen.bench.batch_gemm_bench > $O/sweep.jsonl 2> $O/sweep.err || { tail -5 $O/sweep.err; exit 1; }
python3 -c "
import json
for l in open('$O/sweep.jsonl'):
    d=json.loads(l); print(f\"{d['shape']:8s} M={d['M']:4d} batch {d['batch_us']:7.1f} us ({d['batch_tb_s']:5.2f} TB/s)  hipblaslt {d['hipblaslt_us']:7.1f} us  x{d['speedup']:.2f}  err {d['err_batch']:.3g}/{d['err_hipblaslt']:.3g}\")
"
for v in 1 0; do export LUMEN_BATCH_GEMM=$v;
  LUMEN_BATCH_GEMM=$v timeout -k 10 300 python -m lumen.bench.serve_bench > $O/engine_bg$v.json 2> $O/engine_bg$v.err || { tail -5 $O/engine_bg$v.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/engine_bg$v.json').read().splitlines()[-1]);print('engine batch_gemm=$v', d['output_tok_s'], 'ttft p50', d['ttft_p50_ms'], 'itl p50/p99', d['itl_p50_ms'], d['itl_p99_ms'], 'steps', d['steps'])"
done
