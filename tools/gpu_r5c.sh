#!/bin/bash
# Round 5, call c: the driver's default bench command (erase stage, cfg2 /
# cfg5 riders), timed end to end.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
OUT=gpurun_out/r5c
mkdir -p $OUT
T0=$(date +%s)
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2> $OUT/bench.err
rc=$?; echo "bench exit $rc wall $(( $(date +%s) - T0 )) s"
grep '^{' $OUT/bench.log | python3 tools/summarize_line.py
exit $rc
