#!/bin/bash
# Round 3y: cfg4 A/B -- encoder split into two programs (48 + 36 rows in 6-row
# passes, or 42 + 42 in 7-row passes) against one 84-row program in 11-row
# passes, and the generic reconstruct's row tile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 HBRBC_JIT=load
mkdir -p gpurun_out
SETS="HBRBC_AB_BASE=1 HBRBC_JIT_GROUP=2112,HBRBC_RT_SPEC=6 HBRBC_JIT_GROUP=1848,HBRBC_RT_SPEC=7 HBRBC_RT_REC=7 HBRBC_RT_REC=14 HBRBC_RT_REC=10 HBRBC_AB_BASE=2" CONFIGS=cfg4 STEPS=4 bash tools/ab_env.sh
