#!/bin/bash
# Round 4, call af: the committed profile set at the final cfg3 default
# (32768 instances): kernel trace + stats, FETCH / WRITE / SQ_INSTS_VALU passes
# (tools/pmc_traffic.py -> profiles/pmc_traffic.json, valu_ops_per_perm.json).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
TAG=r4af_cfg3 BENCH_ARGS="--steps 5 --warmup 1 --no-cpu --mode instances --no-leaf-reuse --f4-checks 0" bash tools/profile.sh
