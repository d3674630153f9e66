#!/bin/bash
# Round 6, call n: the microbenchmark with the Miller-step units, then the
# default line on the current code (cfg5 at 4096).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r6n
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 180 ./tools/fp_microbench > $OUT/fp_microbench.jsonl 2>&1
rc=$?; echo "microbench exit $rc"; cat $OUT/fp_microbench.jsonl; if fatal $rc; then exit $rc; fi
export HBRBC_JIT=load
start=$(date +%s)
timeout -k 10 500 python bench.py --detail $OUT/detail.json > $OUT/bench.log 2>&1
rc=$?; echo "bench exit $rc after $(( $(date +%s) - start )) s"; grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json; wc -c $OUT/bench.json
exit $rc
