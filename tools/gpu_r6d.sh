#!/bin/bash
# Round 6, call d: the f4 tower-arithmetic microbenchmark (tools/fp_microbench.hip)
# -- timing, then one SQ_INSTS_VALU pass for lane-ops per unit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6d
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 120 ./tools/fp_microbench > $OUT/fp_microbench.jsonl 2>&1
rc=$?; echo "microbench exit $rc"; cat $OUT/fp_microbench.jsonl; if fatal $rc; then exit $rc; fi
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $OUT/pmc -o run -- ./tools/fp_microbench > $OUT/pmc.log 2>&1
rc=$?; echo "pmc exit $rc"
exit 0
