#!/bin/bash
# transposed FA forward: numerics, micro timing for t1/t2/old, training bench
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -m gpu -k "flash or transpose or llama" > gpurun_out/r14_tests.log 2>&1 || { tail -40 gpurun_out/r14_tests.log; exit 1; }
tail -2 gpurun_out/r14_tests.log
for f in old t1 t2; do
  LUMEN_FA_FWD=$f timeout -k 10 200 python lumen/bench/attn_bench.py --only fwd > gpurun_out/r14_attn_$f.log 2>&1 || { cat gpurun_out/r14_attn_$f.log; exit 1; }
  echo "== $f"; grep -v amdgpu.ids gpurun_out/r14_attn_$f.log
done
LUMEN_FA_FWD=t1 timeout -k 10 200 python lumen/bench/attn_bench.py --only fwd --B 1 --S 4096 > gpurun_out/r14_attn_long.log 2>&1 && grep -v amdgpu.ids gpurun_out/r14_attn_long.log
LUMEN_FA_FWD=t2 timeout -k 10 200 python lumen/bench/attn_bench.py --only fwd --B 1 --S 4096 >> gpurun_out/r14_attn_long.log 2>&1 && tail -3 gpurun_out/r14_attn_long.log
for f in t1 t2; do
  LUMEN_FA_FWD=$f timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/r14_bench_$f.log 2>&1 || exit $?
  echo "$f: $(grep -h '^{' gpurun_out/r14_bench_$f.log | cut -c100-200)"
done
