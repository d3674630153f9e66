#!/bin/bash
# Round 4, call f: the committed profile set of the default cfg3 line --
# kernel trace + stats with the bench line it agrees with, the FETCH / WRITE
# / SQ_INSTS_VALU passes (tools/pmc_traffic.py -> profiles/pmc_traffic.json,
# profiles/valu_ops_per_perm.json), and the stall counters of the default
# kernels (tools/pmc_stall.sh).  Each rocprofv3 run is its own pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
TAG=r4_cfg3 BENCH_ARGS="--steps 5 --warmup 1 --no-cpu --mode instances --no-leaf-reuse --f4-checks 0" bash tools/profile.sh
rc=$?; echo "profile exit $rc"; if fatal $rc; then exit $rc; fi
TAG=r4_stall CONFIG=cfg3 bash tools/pmc_stall.sh > /dev/null
rc=$?; echo "stall exit $rc"; cat gpurun_out/pmc_r4_stall/summary.txt
exit $rc
