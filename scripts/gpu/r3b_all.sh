#!/bin/bash
# one call: schedules + 70B + offload (r3b_sched), the compat CLI (r3b_compat), serving profile
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu/r3b_sched.sh && bash scripts/gpu/r3b_compat.sh && bash scripts/gpu/r3b_serveprof.sh
