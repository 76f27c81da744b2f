#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu/r5_04.sh && bash scripts/gpu/r5_03.sh
