#!/bin/bash
# round-3 closing measurements: default bench (train + extra.serve), bf16 vs fp16 same box,
# forced-partition keep, serving engine + HTTP, reference-compatible ZeRO-3 CLI
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3c_final}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20; tail -1 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
summ() { python3 -c "import json;d=json.load(open('$1'));e=d['extra'];print('$2', d['ms_per_step'], 'ms/step', d['value'], 'tok/s', 'peak GB', e['peak_hbm_gb_max_rank'], 'sched', (e['zero3'] or {}).get('schedule'), 'serve', (e.get('serve') or {}).get('output_tok_s'))"; }
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
summ $O/bench_default.json default
timeout -k 10 300 python bench.py --no_serve --steps 20 --warmup 5 > $O/bf16.json 2> $O/bf16.err || { tail -5 $O/bf16.err; exit 1; }
summ $O/bf16.json bf16
timeout -k 10 300 python bench.py --no_serve --dtype fp16 --steps 20 --warmup 5 > $O/fp16.json 2> $O/fp16.err || { tail -5 $O/fp16.err; exit 1; }
summ $O/fp16.json fp16
# fp16 whole-wave split parts of the gate|up forward (20480 + 1536 columns): tune, then re-measure
LUMEN_TUNE_ROTATING_MB=0 timeout -k 10 600 python -m lumen.bench.split_gemm_probe --dtype fp16 --tune $O/table_fp16.csv > $O/tune16.log 2>&1 || { tail -5 $O/tune16.log; exit 1; }
grep -c Half $O/table_fp16.csv
LUMEN_GEMM_TABLE=$O/table_fp16.csv timeout -k 10 300 python bench.py --no_serve --dtype fp16 --steps 20 --warmup 5 > $O/fp16_split.json 2> $O/fp16_split.err || { tail -5 $O/fp16_split.err; exit 1; }
summ $O/fp16_split.json fp16_split
LUMEN_ZERO3_SINGLE=1 timeout -k 10 300 python bench.py --no_serve --steps 20 --warmup 5 > $O/keep_forced.json 2> $O/keep_forced.err || { tail -5 $O/keep_forced.err; exit 1; }
summ $O/keep_forced.json keep_forced
timeout -k 10 400 python -m lumen.bench.serve_bench --mode http > $O/http.json 2> $O/http.err || { tail -5 $O/http.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/http.json').read().splitlines()[-1]);print('http', d['output_tok_s'], 'ttft p50', d['ttft_p50_ms'], 'itl p50/p99', d['itl_p50_ms'], d['itl_p99_ms'])"
timeout -k 10 400 python training/train_deepspeed_zero3.py --deepspeed configs/ds_config_zero3_mi355x.json \
    --synthetic --synthetic_samples 512 --max_steps 24 --logging_steps 8 --save_strategy no \
    --output_dir /tmp/ck_fused --metrics_csv /tmp/m_fused.csv > $O/zero3_cli.log 2>&1 || { tail -20 $O/zero3_cli.log; exit 1; }
grep -E "window_tokens" $O/zero3_cli.log | tail -1 | cut -c1-300
