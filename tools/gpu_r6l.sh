#!/bin/bash
# Round 6, call l: kernel trace of cfg5 at its new batch (4096), then the
# default line (cfg5 rider at 4096, the pipelines' dominant-stage fix).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HBRBC_JIT=load
ROOT=$PWD
OUT=gpurun_out/r6l
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_cfg5 -o run -- python3 $ROOT/bench.py --config cfg5 --steps 5 --warmup 1 --no-cpu --mode instances --no-leaf-reuse --f4-checks 0 --no-riders > $OUT/trace_cfg5.log 2>&1
rc=$?; echo "trace cfg5 exit $rc"; grep '^{' $OUT/trace_cfg5.log | tail -1 > $OUT/trace_cfg5_bench.json
if fatal $rc; then exit $rc; fi
/usr/bin/time -v timeout -k 10 500 python bench.py --detail $OUT/detail.json > $OUT/bench.log 2> $OUT/bench.err
rc=$?; echo "bench exit $rc"; grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json; wc -c $OUT/bench.json; grep -E "Elapsed|Maximum resident" $OUT/bench.err
exit $rc
