#!/bin/bash
# rocprofv3 kernel stats (CSV) of the 1-GPU training bench: s4_prof.sh OUT
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s4_prof}; mkdir -p $O
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 $O/prof.log | cut -c1-200
find $O/prof -name "*stats*" | head; rm -f $(find $O/prof -name "*kernel_trace.csv"); exit $rc
