#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3_gcheck}; mkdir -p $O
T=configs/tunableop/mi355x_gemms.csv
sed "s/^\(GemmTunableOp_BFloat16_TN,tn_4096_4096_22016_ld_22016_22016_4096,\)[^,]*,/\1Gemm_Hipblaslt_627945,/" $T > $O/t_gu_dx.csv
timeout -k 10 120 python -m lumen.bench.gemm_check $T 4096 4096 22016 2>&1 | grep max_err || exit 1
timeout -k 10 120 python -m lumen.bench.gemm_check $O/t_gu_dx.csv 4096 4096 22016 2>&1 | grep -E "max_err|Error" || exit 1
