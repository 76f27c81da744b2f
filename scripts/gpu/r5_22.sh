#!/bin/bash
# serving projections with the whole-wave split: GPU test, mixed-step probe and chunked engine A/B (split on / off)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5_22; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "wave_split" > $O/test.txt 2>&1 || { tail -20 $O/test.txt; exit 1; }
tail -1 $O/test.txt
for v in 1 0 1 0; do
  LUMEN_GEMM_SPLIT=$v timeout -k 10 300 python -u scripts/probes/mixed_step_probe.py >> $O/mixed_split$v.txt 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
done
for v in 1 0; do grep ms_per $O/mixed_split$v.txt | sed "s/^/split=$v /"; done
for v in 1 0 1 0; do
  LUMEN_GEMM_SPLIT=$v timeout -k 10 400 python -u -m lumen.bench.serve_bench --mode engine --max-model-len 1024 --scheduling-policy chunked --max-batched-tokens 2048 > $O/chunked_split$v.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  echo "split=$v $(python3 -c "import json;d=[json.loads(l) for l in open('$O/chunked_split$v.json') if l.startswith('{')][-1];print(d.get('output_tok_s'), d.get('itl_p99_ms'))")"
done
for v in 1 0 1 0; do
  LUMEN_GEMM_SPLIT=$v timeout -k 10 400 python -u -m lumen.bench.serve_bench --mode engine --max-model-len 1024 --scheduling-policy prefill_first --max-batched-tokens 4096 > $O/pf_split$v.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  echo "prefill_first split=$v $(python3 -c "import json;d=[json.loads(l) for l in open('$O/pf_split$v.json') if l.startswith('{')][-1];print(d.get('output_tok_s'), d.get('itl_p99_ms'))")"
done
