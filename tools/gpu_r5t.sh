#!/bin/bash
# Round 5, call t: per-round kernel trace and SQ counters of the state
# machine after the sender-loop rework (sm_bench, default launch forms).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT_DIR=$ROOT/hbbft_amd/jit
OUT=gpurun_out/r5t
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/trace -o run -- python3 $ROOT/tools/sm_bench.py --reps 3 > $ROOT/$OUT/trace.log 2>&1
rc=$?; echo "trace exit $rc"; if fatal $rc; then exit $rc; fi
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_BRANCH --output-format csv -d $ROOT/$OUT/pmc -o run -- python3 $ROOT/tools/sm_bench.py --reps 1 > $ROOT/$OUT/pmc.log 2>&1
rc=$?; echo "pmc exit $rc"
exit $rc
