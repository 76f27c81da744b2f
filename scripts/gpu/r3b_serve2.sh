#!/bin/bash
# GPU suite; serving A/B of overlapped mixed steps (engine) + HTTP; compat CLI with fused
# accumulation; default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3b_serve2}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20; tail -1 $O/gpu_tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for ov in 1 0; do
  LUMEN_SERVE_OVERLAP=$ov timeout -k 10 300 python -m lumen.bench.serve_bench > $O/engine_ov$ov.json 2> $O/engine_ov$ov.err || { tail -5 $O/engine_ov$ov.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/engine_ov$ov.json').read().splitlines()[-1]);print('engine overlap=$ov', d['output_tok_s'], 'ttft p50', d['ttft_p50_ms'], 'itl p50/p99', d['itl_p50_ms'], d['itl_p99_ms'], 'steps', d['steps'])"
done
timeout -k 10 400 python -m lumen.bench.serve_bench --mode http > $O/http.json 2> $O/http.err || { tail -5 $O/http.err; exit 1; }
python -c "import json;d=json.loads(open('$O/http.json').read().splitlines()[-1]);print('http', d['output_tok_s'], 'ttft p50', d['ttft_p50_ms'], 'itl p50/p99', d['itl_p50_ms'], d['itl_p99_ms'])"
timeout -k 10 400 python training/train_deepspeed_zero3.py --deepspeed configs/ds_config_zero3_mi355x.json \
    --synthetic --synthetic_samples 512 --max_steps 24 --logging_steps 8 --save_strategy no \
    --output_dir /tmp/ck_fused --metrics_csv /tmp/m_fused.csv > $O/zero3_default_fused.log 2>&1 || { tail -20 $O/zero3_default_fused.log; exit 1; }
grep -E "activation checkpointing|window_tokens" $O/zero3_default_fused.log | tail -2 | cut -c1-300
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['ms_per_step'], d['value']);print('serve', d['extra']['serve'])"
