#!/bin/bash
# first GPU pass: kernel numerics, smoke, short bench (each step time-limited; stop on fault)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
python -c "import torch;print(torch.cuda.get_device_name(0))" > gpurun_out/dev.log 2>&1
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/kernels.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench1.log 2>&1
rc=$?
echo "bench rc=$rc"
exit $rc
