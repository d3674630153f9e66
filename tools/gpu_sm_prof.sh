#!/bin/bash
# Kernel trace of the validator-sharded bench objects (state machine rounds).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-smprof}
OUT=$PWD/gpurun_out/prof_$TAG
mkdir -p $OUT
HBRBC_JIT=load timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --mode both --steps 3 --warmup 1 --f4-checks 0 --no-cpu ${BENCH_ARGS} > $OUT/trace.log 2>&1
rc=$?; echo "trace exit $rc"
f=$(find $OUT -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -40 $f
exit $rc
